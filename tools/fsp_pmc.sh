# SQ counters of the chunk decoder (k_fsp_decode) on a 64 MiB zlib stream
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fsp_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export SIZE=$((64<<20))
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/p1" -o run --output-format csv -- python3 "$R/tools/fsp_rate.py" > "$OUT/p1.log" 2>&1 || { echo p1 failed; tail -5 "$OUT/p1.log"; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU -d "$OUT/p2" -o run --output-format csv -- python3 "$R/tools/fsp_rate.py" > "$OUT/p2.log" 2>&1 || { echo p2 failed; tail -5 "$OUT/p2.log"; exit 3; }
echo ok
