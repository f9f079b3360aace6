"""Run one of the reference's scripts (train_vit.py, eval_vit.py, ...) on this build's modules.

    python visiontransformer-intention-prediction_amd/run_with_ivit.py /path/to/reference/train_vit.py [args]

``python script.py`` puts the script's own directory at ``sys.path[0]``, ahead of PYTHONPATH,
so ``PYTHONPATH=<pkg> python reference/train_vit.py`` would still import the reference's own
``model_vit`` / ``loss`` / ``utils``. This launcher builds the path itself — this package
first, then the script's directory (for the modules the build does not provide: ``dataset``,
``heuristic_labeling``, ...), then the rest — and executes the script with ``runpy`` as
``__main__`` (runpy.run_path on a file does not touch ``sys.path``). Modules that both provide
(``model_vit``, ``heads``, ``loss``, ``utils``, ``constants``, ``model_cnn``) resolve to the build.
"""
from __future__ import annotations

import os
import runpy
import sys

PKG = os.path.dirname(os.path.abspath(__file__))


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        raise SystemExit(__doc__)
    script = os.path.abspath(argv[0])
    sdir = os.path.dirname(script)
    here = os.path.abspath(os.getcwd())
    rest = [p for p in sys.path if os.path.abspath(p or here) not in (PKG, sdir)]
    sys.path[:] = [PKG, sdir] + rest
    sys.argv = [script] + argv[1:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
