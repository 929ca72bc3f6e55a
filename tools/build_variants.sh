#!/bin/bash
# A/B builds of libminisched_gpu.so with extra -D flags on ms_kernels.hip, for
# MINISCHED_LIB=... runs (tools/gpu_*.sh). Usage: tools/build_variants.sh NAME "-DFOO=1 ..." [vst]
# -> mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_NAME.so (vst: with the MS_VSTAMPS stamps;
# tl: the per-workgroup step timeline only, e.g. tools/build_variants.sh tl "" tl)
set -e
cd "$(dirname "$0")/../mini-kube-scheduler_amd"
NAME=$1; DEFS=$2; VST=$3
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I../include -Icsrc"
mkdir -p build
if [ "$VST" = vst ]; then
  $H -DMS_VSTAMPS $DEFS -c csrc/ms_kernels.hip -o build/ms_kernels_$NAME.o
  $H -DMS_VSTAMPS $DEFS -c csrc/ms_capi.cpp -o build/ms_capi_vst_$NAME.o  # (host-side -D flags too)
  CAPI=build/ms_capi_vst_$NAME.o
elif [ "$VST" = tl ]; then  # step timeline only (MS_TIMELINE=<file>; the host side reads it since round 6)
  $H -DMS_TIMELINE_ONLY $DEFS -c csrc/ms_kernels.hip -o build/ms_kernels_$NAME.o
  $H -DMS_TIMELINE_ONLY $DEFS -c csrc/ms_capi.cpp -o build/ms_capi_tl_$NAME.o
  CAPI=build/ms_capi_tl_$NAME.o
else
  $H $DEFS -c csrc/ms_kernels.hip -o build/ms_kernels_$NAME.o
  CAPI=build/ms_capi.o
  if [ -n "$DEFS" ]; then  # (host-side constants such as MS_WARM_PODS take the same -D flags)
    $H $DEFS -c csrc/ms_capi.cpp -o build/ms_capi_$NAME.o
    CAPI=build/ms_capi_$NAME.o
  fi
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o minisched_amd/libminisched_gpu_$NAME.so build/ms_kernels_$NAME.o build/ms_sweep_pp.o build/ms_taint.o build/ms_affinity.o $CAPI build/ms_comm.o -L/opt/rocm/lib -lrccl
echo built minisched_amd/libminisched_gpu_$NAME.so
