#!/bin/bash
# dev A/B: build variant libraries: tools/variants.sh build NAME "EXTRA flags" ...
#          then on the GPU: tools/variants.sh run NAME ...
R=$(cd "$(dirname "$0")/.." && pwd)
cmd=$1; shift
if [ "$cmd" = build ]; then
    while [ $# -gt 0 ]; do
        n=$1; f=$2; shift 2
        make -s -C $R/jdeflate_amd/csrc OUT=$R/tools/var/$n OBJ=$R/tools/var/$n/obj EXTRA="$f" $R/tools/var/$n/libjdeflate_amd.so || exit 1
    done
else
    mkdir -p $R/gpurun_out
    for n in "$@"; do
        echo "== $n"
        JDAMD_LIB=$R/tools/var/$n/libjdeflate_amd.so timeout -k 10 300 python3 $R/tools/probe.py || exit 1
    done
fi
