#!/bin/bash
# One parameterised GPU-box runner (replaces the per-run gpu_r04*.sh scripts).
# Each STEP runs under its own time limit; the first failure ends the call.
# Outputs go to gpurun_out/<TAG>_<step>*.
#
#   bash tools/gpu.sh TAG STEP [STEP ...]
#
# STEP (arguments separated by '|'):
#   tests[|<pytest -k expr>]            product library, pytest -m gpu
#   devtests|<ENV=V,...>[|<-k expr>]    the GPU suite on libsyncr_cdc_dev.so with a variant forced
#   smoke                               __graft_entry__.smoke()
#   bench[|<extra bench.py flags>[|<checkout>[|<ENV=V,...>]]]  the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   ab|<workload>|<rounds>[e]|<V1>|<V2>... tools/dip_ab.py variants (dev library) in the driver's condition
#                                       (rounds suffix e: scan timed by HIP events)
#   trace|<workload>[|<shard>[|--no-events[|<checkout>]]]  kernel trace of one small-batch leg
#                                       (tools/legs_trace.py, product; <checkout>: e.g. build/r04src)
#   pmc|<workload>|<counters>          one rocprofv3 --pmc pass over a legs_trace.py leg (per-kernel means)
#   sttrace|<workload>|<ENV=V,...>      per-wave stream-tile scan timeline (tools/scan_timeline.py, dev)
#   restl|<workload>                    resolve timeline (tools/resolve_timeline.py, dev library)
#   prof|<PROFTAG>[|<extra flags>[|<ENV=V,...>]]  tools/prof.sh: trace + traffic + SQ passes of the driver's
#                                       command (e.g. "prof|r05_st18|--dev-lib|SYNCR_CDC_ST_SEGS=18")
#   rehearse|<N>                        torch.distributed.run with N ranks, all on device 0 (a flow check)
#   e2etrace|<mode>|<files>             benchlib/e2e_driver.cpp <mode> over the first <files> zipf10k files,
#                                       under rocprofv3 --kernel-trace --hip-trace --stats
#   e2eab|<libdirs,>[|<modes,>[|<rounds>]]  tools/e2e_ab.py: e2e_driver legs against several library builds,
#                                       interleaved (e.g. "e2eab|syncr_amd,build/ab_pre/syncr_amd")
#   build                               python -m syncr_amd.build (+ --dev) on the box (normally built here)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
TAG=$1
shift
export TMPDIR=/tmp

envrun() {   # envrun "A=1,B=2" cmd...: run cmd with the comma-separated variables set
    local kv=$1; shift
    ( IFS=','; for x in $kv; do [ -n "$x" ] && export "$x"; done; "$@" )
}

n=0
for step in "$@"; do
    n=$((n + 1))
    IFS='|' read -r -a a <<< "$step"
    kind=${a[0]}
    out="$O/${TAG}_${n}_${kind}"
    echo "== step $n: $step"
    case "$kind" in
    tests)
        K=(); [ -n "${a[1]}" ] && K=(-k "${a[1]}")
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$out.log" 2>&1 \
            || { echo "tests failed rc=$?"; tail -40 "$out.log"; exit 11; }
        tail -2 "$out.log" ;;
    devtests)
        K=(); [ -n "${a[2]}" ] && K=(-k "${a[2]}")
        envrun "SYNCR_TEST_DEV_LIBRARY=1,${a[1]}" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
            --timeout-method thread "${K[@]}" > "$out.log" 2>&1 || { echo "devtests failed rc=$?"; tail -40 "$out.log"; exit 12; }
        tail -2 "$out.log" ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out.log" 2>&1 \
            || { echo "smoke failed rc=$?"; tail -20 "$out.log"; exit 13; }
        tail -c 300 "$out.log"; echo ;;
    bench)
        BROOT=$R/${a[2]:-.}                         # another checkout's bench (e.g. build/r04src: same-box A/B)
        ( cd "$BROOT" && envrun "${a[3]}" timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${a[1]} ) > "$out.json" \
            2> "$out.err" || { echo "bench failed rc=$?"; tail -30 "$out.err"; exit 14; }
        python tools/bench_summary.py "$out.json" ;;
    ab)
        EV=(); [[ "${a[2]}" == *e ]] && EV=(--events)          # rounds "4e": HIP-event scan timing
        timeout -k 10 600 python -u tools/dip_ab.py "${a[@]:3}" --workload "${a[1]}" --rounds "${a[2]%e}" "${EV[@]}" > "$out.jsonl" 2> "$out.err" \
            || { echo "ab failed rc=$?"; tail -30 "$out.err"; exit 15; }
        python - "$out.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["workload"], {v: (x["scan_ms_med"], x["step_ms_med"]) for v, x in d["variants"].items()})
PY
        ;;
    trace)
        P=$O/${TAG}_${n}_trace_${a[1]}
        mkdir -p "$P"
        SH=${a[2]:-0}
        LROOT=$R/${a[4]:-.}                        # another checkout's leg (e.g. build/r04src: before/after)
        ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$P" -o run -- \
            python3 "$LROOT/tools/legs_trace.py" --workload "${a[1]}" --shard "$SH" ${a[3]} > "$P/leg.json" 2> "$P/leg.err" ) \
            || { echo "trace failed rc=$?"; tail -20 "$P/leg.err"; exit 16; }
        f=$(find "$P" -name '*kernel_trace.csv' | head -1)
        nb=$(python3 -c "import json;print(json.loads(open('$P/leg.json').read().strip().splitlines()[-1])['bytes'])")
        python3 tools/legs_trace_show.py "$f" 20 5 "$nb" > "$P/steps.json" && cat "$P/steps.json" | head -30 ;;
    pmc)                                         # pmc|<workload>|<counters, space-separated>: one PMC pass
        P=$O/${TAG}_${n}_pmc_${a[1]}
        mkdir -p "$P"
        ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc ${a[2]} --output-format csv -d "$P" -o run -- \
            python3 "$R/tools/legs_trace.py" --workload "${a[1]}" --steps 5 --warmup 2 > "$P/leg.json" 2> "$P/leg.err" ) \
            || { echo "pmc failed rc=$?"; tail -20 "$P/leg.err"; exit 21; }
        f=$(find "$P" -name '*counter_collection.csv' | head -1)
        python3 tools/pmc_kernels.py "$f" > "$P/kernels.json" && cat "$P/kernels.json" ;;
    sttrace)
        envrun "${a[2]}" timeout -k 10 300 python -u tools/scan_timeline.py --workload "${a[1]}" > "$out.json" 2> "$out.err" \
            || { echo "sttrace failed rc=$?"; tail -20 "$out.err"; exit 17; }
        head -c 1500 "$out.json"; echo ;;
    restl)
        timeout -k 10 300 python -u tools/resolve_timeline.py --workload "${a[1]}" --launches 3 > "$out.txt" 2> "$out.err" \
            || { echo "restl failed rc=$?"; tail -20 "$out.err"; exit 20; }
        cat "$out.txt" ;;
    prof)
        envrun "${a[3]}" bash tools/prof.sh "${a[1]}" ${a[2]} || { echo "prof failed rc=$?"; exit 18; } ;;
    rehearse)                                  # rehearse|N: the driver's N-rank launcher, every rank on device 0
        N=${a[1]:-2}
        DM=$(python3 -c "print(','.join(['0']*$N))")
        timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
            --master-port $((29500 + N)) bench.py --gpus "$N" --steps 20 --warmup 5 --device-map "$DM" > "$out.json" \
            2> "$out.err" || { echo "rehearse failed rc=$?"; tail -30 "$out.err"; exit 22; }
        python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('n_gpus', d['n_gpus'], 'value', d['value'], d.get('load_balance'), d['parity'].get('headline'))" "$out.json" ;;
    e2etrace)                                  # e2etrace|<mode>|<files>: one e2e_driver mode under the kernel + HIP API trace
        P=$O/${TAG}_${n}_e2etrace_${a[1]}
        mkdir -p "$P"
        timeout -k 10 300 python3 tools/e2e_tree.py /tmp/syncr_e2e_tree --files "${a[2]:-500}" > "$P/tree.log" 2>&1 || { echo "tree failed"; exit 23; }
        python3 -c "from benchlib import e2e; e2e.driver()" || exit 23
        ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d "$P" -o run -- \
            "$R/build/e2e_driver" "${a[1]}" /tmp/syncr_e2e_tree "$P/results.bin" --reps 1 > "$P/driver.json" 2> "$P/driver.err" ) \
            || { echo "e2etrace failed rc=$?"; tail -20 "$P/driver.err"; exit 24; }
        rm -rf /tmp/syncr_e2e_tree "$P/results.bin"
        cat "$P/driver.json"; head -12 "$P"/*kernel_stats.csv; head -15 "$P"/*hip_api_stats.csv 2>/dev/null ;;
    e2eab)
        timeout -k 10 900 python -u tools/e2e_ab.py --libs "${a[1]}" --modes "${a[2]:-files,mem,zero_copy,walk}" \
            --rounds "${a[3]:-3}" > "$out.jsonl" 2> "$out.err" || { echo "e2eab failed rc=$?"; tail -20 "$out.err"; exit 25; }
        tail -1 "$out.jsonl" ;;
    build)
        timeout -k 10 900 python -m syncr_amd.build --force > "$out.log" 2>&1 && \
        timeout -k 10 900 python -m syncr_amd.build --force --dev >> "$out.log" 2>&1 || { echo "build failed"; exit 19; } ;;
    *)
        echo "unknown step $kind"; exit 2 ;;
    esac
done
echo "gpu.sh $TAG: all steps done"
