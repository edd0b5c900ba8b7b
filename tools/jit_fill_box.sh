#!/bin/bash
# Compile the query-specialised NFA kernels of tools/jit_precompile.py on the GPU box into siddhi_amd/jit_cache (the
# box's hiprtc: kernels built on the CPU-only build host came out with 256 VGPRs and 192 B of scratch where the box's
# build of the same source and options has 170 and 112 B, and ran 4 % slower), copy them to gpurun_out/jc for the
# tree, then run NFA parity (ARGS: extra tools/step.sh steps).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/jc
echo "hiprtc: $(ls -l /opt/rocm/lib/libhiprtc.so* 2>&1 | tr '\n' ' ') rocm $(cat /opt/rocm/.info/version 2>/dev/null)"
timeout -k 10 600 env SM_NFA_JIT_COMPACT=1 python -u tools/jit_precompile.py -j 8 || exit 1
cp siddhi_amd/jit_cache/*.co gpurun_out/jc/ || exit 1
ls -l gpurun_out/jc
