#!/bin/bash
# One launcher for every GPU measurement of a round (replaces the per-call scripts).
#   bash tools/gpu.sh TAG STEP [STEP ...]        (run through gpurun, from the repo root)
# Output goes to gpurun_out/TAG/.  Steps (each under its own time limit; the chain
# stops at the first step that faults, aborts, times out or fails):
#   suite          pytest -m gpu (one process)            -> suite.txt
#   suite:EXPR     the same restricted to -k EXPR
#   smoke          __graft_entry__.smoke()                 -> smoke.txt
#   bench          python bench.py (headline, cpu baseline) -> bench_nlse3d_512.json
#   bench:WL       python bench.py --workload WL            -> bench_WL.json
#   set            bench of every BASELINE workload + KG    -> bench_*_set.json
#   prof[:WL]      bench under rocprofv3 --kernel-trace --stats -> prof_WL/, bench_WL_under_rocprof.json
#   pmc[:WL]       FETCH_SIZE / WRITE_SIZE / TCC hit passes, one counter group per run -> pmc_WL/
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (a probe)           -> py_<name>.txt
set -o pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # run LIMIT OUTFILE CMD...: stop the chain on any failure
  local lim=$1 out=$2
  shift 2
  echo "[gpu.sh] $(date +%T) $*"
  timeout -k 10 "$lim" "$@" > "$out" 2> "$out.err"
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "[gpu.sh] '$*' exited $rc; stopping" >&2
    tail -n 20 "$out" >&2
    tail -n 20 "$out.err" >&2
    exit $rc
  fi
}
for st in "$@"; do
  name=${st%%:*}
  arg=""
  [ "$name" != "$st" ] && arg=${st#*:}
  case $name in
    suite)
      if [ -n "$arg" ]; then
        run 900 "$OUT/suite.txt" python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$arg"
      else
        run 900 "$OUT/suite.txt" python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
      fi
      tail -3 "$OUT/suite.txt" ;;
    suitev)
      # suitev:VARIANT:EXPR -- the GPU tests matching EXPR against nonlinear-solvers_amd/VARIANT
      v=${arg%%:*}
      ex=${arg#*:}
      NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/$v/libnls_amd.so run 900 "$OUT/suite_$v.txt" \
        python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$ex"
      tail -n 3 "$OUT/suite_$v.txt" ;;
    smoke)
      run 180 "$OUT/smoke.txt" python -c "import __graft_entry__ as g; g.smoke()"
      cat "$OUT/smoke.txt" ;;
    bench)
      if [ -n "$arg" ]; then
        run 300 "$OUT/bench_$arg.json" python bench.py --workload "$arg" --no-cpu-baseline
        cat "$OUT/bench_$arg.json"
      else
        run 300 "$OUT/bench_nlse3d_512.json" python bench.py
        cat "$OUT/bench_nlse3d_512.json"
      fi ;;
    set)
      for w in nlse2d_4096 sg2d_8192 g2_3d_256 kg_3d_256 cq3d_1024 nlse3d_512; do
        run 300 "$OUT/bench_${w}_set.json" python bench.py --workload "$w" --steps 10 --warmup 2 --no-cpu-baseline
        cat "$OUT/bench_${w}_set.json"
      done ;;
    prof)
      wl=${arg:-nlse3d_512}
      run 300 "$OUT/bench_${wl}_under_rocprof.json" rocprofv3 --kernel-trace --stats -d "$OUT/prof_$wl" -o run \
        --output-format csv -- python3 bench.py --workload "$wl" --steps 10 --warmup 2 --no-cpu-baseline
      # the bench's own dispatches (after the placement probe's; tools/trace_stats.py)
      f=$(ls "$OUT/prof_$wl"/*kernel_trace.csv 2>/dev/null | head -n 1)
      [ -n "$f" ] && python3 tools/trace_stats.py "$f" > "$OUT/prof_$wl/bench_kernel_stats.csv"
      cat "$OUT/bench_${wl}_under_rocprof.json" ;;
    pmc)
      wl=${arg:-nlse3d_512}
      i=0
      mkdir -p "$OUT/pmc_$wl"
      for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
        i=$((i + 1))
        echo "[gpu.sh] $(date +%T) pmc $grp"
        # NLS_PLACE=1: no placement probe (its candidates' dispatches would enter the per-kernel
        # averages; the bytes a kernel moves do not depend on the placement,
        # profiles/r06/place_diag.txt), so the tails that write u stay 2 of 7
        NLS_PLACE=1 timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$wl/p$i" -o run -- \
          python3 bench.py --workload "$wl" --steps 2 --warmup 0 --no-cpu-baseline > "$OUT/pmc_$wl/p$i.log" 2>&1 || exit $?
      done ;;
    sq)
      # issue / wait fractions and instruction counts per wave (8 SQ counters, one pass)
      wl=${arg:-nlse3d_512}
      mkdir -p "$OUT/sq_$wl"
      echo "[gpu.sh] $(date +%T) sq $wl"
      NLS_PLACE=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$OUT/sq_$wl/p1" -o run -- \
        python3 bench.py --workload "$wl" --steps 2 --warmup 0 --no-cpu-baseline > "$OUT/sq_$wl/p1.log" 2>&1 || exit $?
      python3 tools/pmc_table.py "$OUT/sq_$wl" > "$OUT/sq_$wl.txt" && cat "$OUT/sq_$wl.txt" ;;
    sq2)
      # LDS and instruction-wait detail (8 SQ counters, one pass)
      wl=${arg:-nlse3d_512}
      mkdir -p "$OUT/sq2_$wl"
      echo "[gpu.sh] $(date +%T) sq2 $wl"
      NLS_PLACE=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
        SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/sq2_$wl/p1" -o run -- \
        python3 bench.py --workload "$wl" --steps 2 --warmup 0 --no-cpu-baseline > "$OUT/sq2_$wl/p1.log" 2>&1 || exit $?
      python3 tools/pmc_table.py "$OUT/sq2_$wl" > "$OUT/sq2_$wl.txt" && cat "$OUT/sq2_$wl.txt" ;;
    ab)
      # same-box A/B: every variant build nonlinear-solvers_amd/lib_v*/ against lib, two
      # rounds interleaved, one bench process each -> ab_WL.txt (ms/step, dominant kernel ms)
      wl=${arg:-nlse3d_512}
      vars=$(cd nonlinear-solvers_amd && ls -d lib_v* 2>/dev/null | tr '\n' ' ')
      for rep in 1 2; do
        for v in $vars lib; do
          NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/$v/libnls_amd.so run 300 "$OUT/ab_${wl}_${v}_$rep.json" \
            python bench.py --workload "$wl" --steps 10 --warmup 2 --no-cpu-baseline
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; k=d['step_roofline']['gpu_kernel_ms_per_step']; \
print(f\"$v rep$rep ms/step {d['ms_per_step']:.3f} value {d['value']:.1f} dominant {r['avg_launch_ms']:.4f} ms frac {r['frac']:.3f} \
\" + ' '.join(f'{a}:{b:.3f}' for a, b in k.items()))" "$OUT/ab_${wl}_${v}_$rep.json" \
            | tee -a "$OUT/ab_$wl.txt"
        done
      done ;;
    p2ab)
      # per-pass times (tools/p2_probe.py, 512^3 m=16) of every lib_v* variant and lib,
      # once per environment setting of the comma list ARG ("-" = none, e.g.
      # "-,NLS_P2_KZJ=16") -> p2ab.txt
      vars=$(cd nonlinear-solvers_amd && ls -d lib_v* 2>/dev/null | tr '\n' ' ')
      for ev in $(echo "${arg:--}" | tr ',' ' '); do
        for rep in 1 2; do
          for v in $vars lib; do
            echo "== $v $ev rep$rep" >> "$OUT/p2ab.txt"
            [ "$ev" != "-" ] && export "${ev?}"
            NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/$v/libnls_amd.so run 300 "$OUT/p2ab_cur.txt" python -u tools/p2_probe.py 512 16 4
            [ "$ev" != "-" ] && unset "${ev%%=*}"
            cat "$OUT/p2ab_cur.txt" >> "$OUT/p2ab.txt"
          done
        done
      done
      cat "$OUT/p2ab.txt" ;;
    envab)
      # same-box A/B of environment settings on one workload: ARG = WL:SET,SET,... ("-" =
      # none), two interleaved rounds (ENVAB_REPS) -> envab_WL.txt
      wl=${arg%%:*}
      sets=${arg#*:}
      for rep in $(seq 1 "${ENVAB_REPS:-2}"); do
        for ev in $(echo "$sets" | tr ',' ' '); do
          # a setting is one VAR=VALUE or several joined by '+'
          [ "$ev" != "-" ] && for kv in $(echo "$ev" | tr '+' ' '); do export "${kv?}"; done
          run 300 "$OUT/envab_cur.json" python bench.py --workload "$wl" --steps 10 --warmup 2 --no-cpu-baseline
          [ "$ev" != "-" ] && for kv in $(echo "$ev" | tr '+' ' '); do unset "${kv%%=*}"; done
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['step_roofline']['gpu_kernel_ms_per_step']; \
print(f\"$ev rep$rep ms/step {d['ms_per_step']:.3f} value {d['value']:.1f} \" + ' '.join(f'{a}:{b:.3f}' for a, b in k.items()) + ' place:' + str(d.get('placement')))" \
            "$OUT/envab_cur.json" | tee -a "$OUT/envab_$wl.txt"
        done
      done ;;
    probe6)
      # pure-stream rates of the tail / pass access patterns (tools/bw_probe6.hip, prebuilt)
      run 300 "$OUT/bw_probe6_512.txt" tools/bw_probe6
      cat "$OUT/bw_probe6_512.txt" ;;
    slab)
      # per-rank cost of the 8-GPU slabs on one GPU (tools/slab_probe.py)
      run 600 "$OUT/slab_probe.txt" python -u tools/slab_probe.py
      cat "$OUT/slab_probe.txt" ;;
    py)
      script=${arg%%:*}
      args=""
      [ "$script" != "$arg" ] && args=${arg#*:}
      # shellcheck disable=SC2086
      run 600 "$OUT/py_$(basename "$script" .py).txt" python -u "$script" $args
      tail -40 "$OUT/py_$(basename "$script" .py).txt" ;;
    *)
      echo "[gpu.sh] unknown step $st" >&2
      exit 2 ;;
  esac
done
echo "[gpu.sh] $(date +%T) done"
