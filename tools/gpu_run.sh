#!/bin/bash
# The one GPU-session runner (run through gpurun from the repo root):
#   bash tools/gpu_run.sh OUT step [step ...]
# steps (each under its own time limit; the session stops at the first step
# that fails, times out or faults):
#   pytest            the whole -m gpu suite
#   pytest:EXPR       -m gpu -k EXPR
#   smoke             __graft_entry__.smoke()
#   bench             python bench.py (the driver's default line)
#   quick             python bench.py --steps 5 --warmup 1 --no-cpu --no-host-api
#   probe             tools/probe.py (per-kernel ms, output CRC)
#   probe:VAR=VAL     the same with an environment switch (e.g. JD_CHAINS_SERIAL=1)
#   var:NAME          tools/probe.py on the variant library tools/var/NAME
#   cnt:VAR=VAL       tools/prof_counters.sh (SQ issue counters) with an env switch
#   mem:VAR=VAL       tools/mem_counters.sh (L1/TA/TD counters) with an env switch
#   mt:VAR=VAL[,..]   tools/mt_rate.py (multi-instance drop-in rate) with env switches
#   sprof             tools/stream_prof.sh (kernel trace of the drop-in stream inflate)
#   collect:TAG       profiles/collect.sh TAG (kernel trace + FETCH/WRITE passes)
#   ab:LIB[,LIB..]    tools/ab_probe.py: per-kernel ms of whole builds, ABBA order
#   rpclock:NAME      tools/rpar_clock.py on an RP_CLOCK build (tools/var/NAME)
#   abmix:LIB[,LIB..] the same on 256 MiB of the mixed corpus at level 9 (C5-like)
#   collectc5:TAG     the same on C5 (4 GiB mixed, level 9) into pmc_summary_c5.json
#   swprobe           tools/sw_probe.py (single-window deflate rate, per-kernel ms)
#   sq:TAG            tools/prof_counters.sh on the bench workload (1 GiB text, L6) ->
#                     gpurun_out/prof_cnt_TAG/sq_summary.json (bench.py's roofline.compute)
#   cpub              tools/cpu_baseline.py (oracle speed on Python source, 1 and 8 threads)
#   overlap           tools/overlap_probe.py (deflate and inflate loops alone / side by side)
#   srate[:NAME]      tools/stream_rate.py (drop-in inflator, 32 KiB reads) [on tools/var/NAME]
#   c5                bench.py on C5 (4 GiB mixed, level 9), 3 steps
# Output: gpurun_out/OUT/<step>.log
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p "$OUT"
cd "$R"
step() {
    local name=$1 lim=$2
    shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc: $(tail -1 "$OUT/$name.log" | cut -c1-300)"
    if [ $rc -ne 0 ]; then
        grep -E "FAILED|Error|error" "$OUT/$name.log" | head -20
        echo "stopping after $name (rc=$rc)"
        exit 1
    fi
}
for s in "$@"; do
    case $s in
        pytest) step pytest 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
        pytest:*) step "pytest_${s#pytest:}" 900 python -u -m pytest tests -m gpu -x -v --timeout 200 \
                       --timeout-method thread -k "${s#pytest:}" ;;
        smoke) step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench 600 python bench.py ;;
        quick) step quick 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-host-api ;;
        probe) step probe 300 python tools/probe.py ;;
        probe:*) env "${s#probe:}" timeout -k 10 300 python tools/probe.py > "$OUT/probe_${s#probe:}.log" 2>&1 \
                     || { echo "probe ${s#probe:} failed"; tail -5 "$OUT/probe_${s#probe:}.log"; exit 1; }
                 echo "probe ${s#probe:}: $(tail -1 "$OUT/probe_${s#probe:}.log" | cut -c1-400)" ;;
        var:*) JDAMD_LIB=$R/tools/var/${s#var:}/libjdeflate_amd.so step "var_${s#var:}" 300 python tools/probe.py ;;
        cnt:*) env "${s#cnt:}" timeout -k 10 600 bash tools/prof_counters.sh "_${s#cnt:}" > "$OUT/cnt_${s#cnt:}.log" 2>&1 \
                   || { echo "cnt ${s#cnt:} failed"; tail -5 "$OUT/cnt_${s#cnt:}.log"; exit 1; }
               echo "cnt ${s#cnt:}: done" ;;
        mem:*) env "${s#mem:}" timeout -k 10 600 bash tools/mem_counters.sh "_${s#mem:}" > "$OUT/mem_${s#mem:}.log" 2>&1 \
                   || { echo "mem ${s#mem:} failed"; tail -5 "$OUT/mem_${s#mem:}.log"; exit 1; }
               echo "mem ${s#mem:}: done" ;;
        mt:*) env $(echo "${s#mt:}" | tr , ' ') timeout -k 10 300 python tools/mt_rate.py > "$OUT/mt_${s#mt:}.log" 2>&1 \
                  || { echo "mt ${s#mt:} failed"; tail -5 "$OUT/mt_${s#mt:}.log"; exit 1; }
              echo "mt ${s#mt:}: $(tail -1 "$OUT/mt_${s#mt:}.log" | cut -c1-400)" ;;
        sprof) step sprof 400 bash tools/stream_prof.sh ;;
        collect:*) step "collect_${s#collect:}" 1000 bash profiles/collect.sh "${s#collect:}" pmc_summary.json ;;
        ab:*) step ab 900 python tools/ab_probe.py $(echo "${s#ab:}" | tr , ' ') ;;
        abmix:*) SIZE=$((256<<20)) LEVEL=9 CORPUS=mixed step abmix 900 python tools/ab_probe.py $(echo "${s#abmix:}" | tr , ' ') ;;
        rpclock:*) JDAMD_LIB=$R/tools/var/${s#rpclock:}/libjdeflate_amd.so step "rpclock_${s#rpclock:}" 600 \
                       python tools/rpar_clock.py ;;
        collectc5:*) step "collectc5_${s#collectc5:}" 1100 bash profiles/collect.sh "${s#collectc5:}" pmc_summary_c5.json \
                         --corpus mixed --level 9 --size 4294967296 ;;
        swprobe) step swprobe 600 python tools/sw_probe.py ;;
        swprobe:*) JDAMD_LIB=$R/tools/var/${s#swprobe:}/libjdeflate_amd.so step "swprobe_${s#swprobe:}" 600 \
                       python tools/sw_probe.py ;;
        cpub) step cpub 600 python tools/cpu_baseline.py ;;
        overlap) step overlap 600 python -u tools/overlap_probe.py ;;
        srate) step srate 300 python tools/stream_rate.py ;;
        srate:*) JDAMD_LIB=$R/tools/var/${s#srate:}/libjdeflate_amd.so step "srate_${s#srate:}" 300 \
                     python tools/stream_rate.py ;;
        sq:*) SIZE=$((1<<30)) SQTAG=${s#sq:} step "sq_${s#sq:}" 900 bash tools/prof_counters.sh "_${s#sq:}" ;;
        c5) step c5 600 python bench.py --corpus mixed --level 9 --size 4294967296 --steps 3 --warmup 1 \
                --no-cpu --no-host-api ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
