#!/bin/bash
# per-kind probe for the in-tree library and each named variant; stops at the first failure
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 $R/tools/kind_probe.py > $R/gpurun_out/kind_tree.log 2>&1 || exit $?
for n in "$@"; do
    JDAMD_LIB=$R/tools/var/$n/libjdeflate_amd.so timeout -k 10 300 python3 $R/tools/kind_probe.py > $R/gpurun_out/kind_$n.log 2>&1 || exit $?
done
