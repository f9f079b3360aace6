#!/bin/bash
# Build libivit_hip.so of a git revision into ab/lib_<name>.so (same-call A/B runs on the GPU box:
# IVIT_LIB=ab/lib_<name>.so python ...).  Usage: tools/ab_build.sh <rev> <name>
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/abbuild.XXXX)
git -C "$ROOT" archive "$REV" | tar -x -C "$T"
make -C "$T/visiontransformer-intention-prediction_amd" -j8 > "$T/make.log" 2>&1
mkdir -p "$ROOT/ab"
cp "$T/visiontransformer-intention-prediction_amd/libivit_hip.so" "$ROOT/ab/lib_$NAME.so"
rm -rf "$T"
echo "built ab/lib_$NAME.so from $REV"
