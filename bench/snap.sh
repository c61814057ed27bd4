#!/bin/bash
# Freeze the working tree (sources + built _C.so) into ./snap for a queued GPU call, so edits made
# while the call waits for a box do not leak into it. GPU commands then run `cd snap && ...`;
# snap/gpurun_out links to the repo's gpurun_out (the only directory gpurun merges back).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -rf snap && mkdir snap
tar --exclude=./.git --exclude=./gpurun_out --exclude=./snap --exclude=./build --exclude='__pycache__' -cf - . | tar -xf - -C snap
ln -sfn ../gpurun_out snap/gpurun_out
