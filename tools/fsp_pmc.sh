# SQ counters of the chunk decoder (k_fsp_decode) on a 64 MiB zlib stream
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fsp_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export SIZE=$((64<<20))
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d "$OUT/p3" -o run --output-format csv -- python3 "$R/tools/fsp_rate.py" > "$OUT/p3.log" 2>&1 || { echo p3 failed; tail -5 "$OUT/p3.log"; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES -d "$OUT/p4" -o run --output-format csv -- python3 "$R/tools/fsp_rate.py" > "$OUT/p4.log" 2>&1 || { echo p4 failed; tail -5 "$OUT/p4.log"; exit 3; }
echo ok
