#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step runs under its own timeout; a crash/timeout (exit >= 124 or signal) ends the
# script immediately.  Test failures (pytest exit 1) do not stop the bench.
# usage: [STEPS="pytest_gpu smoke bench"] tools/gpu_round.sh [tag] [pytest-args...]
# Steps: pytest_gpu smoke bench sweep prof pmc (defaults) and, on request,
#   train_prof  rocprofv3 kernel trace of `bench.py --mode train $TRAIN_ARGS`
#   bench_args  one `bench.py $BENCH_ARGS` line
#   prof_args   rocprofv3 kernel trace of `bench.py $BENCH_ARGS`
#   pmc_args    tools/pmc.sh passes of `bench.py $BENCH_ARGS`, summarised as $PMC_TAG
set -u
STEPS="${STEPS:-pytest_gpu smoke bench sweep prof pmc}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-r01}"; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { echo "FATAL step $1 exit $2"; exit "$2"; }
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  case " $STEPS " in *" $name "*) ;; *) return 0;; esac
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "--- $name exit $rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then fatal "$name" $rc; fi
  return 0
}
rocm-smi --showproductname > "$OUT/rocm-smi.txt" 2>&1 || true
lscpu | grep -E "Model name|^CPU\(s\)" > "$OUT/lscpu.txt" 2>&1 || true
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -x --timeout 200 --timeout-method thread "$@"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 3
# the driver's own command, then the same command under rocprofv3 (kernel trace of the run whose
# line it annotates; tools/prof_vs_line.py windows the trace by each config's timed region)
export GNND_BENCH_FULL="$OUT/bench_default_full.json"
step bench_default 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
export GNND_BENCH_FULL="$OUT/prof_default_full.json"
step prof_default 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_default" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
case " $STEPS " in *" prof_default "*) python tools/prof_vs_line.py "$OUT"/prof_default/run_kernel_trace.csv "$OUT/prof_default_full.json" "$OUT/prof_vs_line.json" > "$OUT/prof_vs_line.txt" 2>&1 || true;; esac
unset GNND_BENCH_FULL
step sweep 900 python tools/sweep.py --steps 5
step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-seconds 0
step pmc 1200 bash tools/pmc.sh "$OUT/pmc"
step train_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/train_prof" -o run --output-format csv -- python bench.py --mode train ${TRAIN_ARGS:-} --cpu-seconds 0
step bench_args 600 python bench.py ${BENCH_ARGS:-}
step prof_args 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_args" -o run --output-format csv -- python bench.py ${BENCH_ARGS:-} --cpu-seconds 0
step pmc_args 1200 bash tools/pmc.sh "$OUT/pmc_args" ${BENCH_ARGS:-}
case " $STEPS " in *" pmc_args "*) python tools/pmc_summary.py "$OUT/pmc_args" "${PMC_TAG:-args}" "$OUT/pmc_${PMC_TAG:-args}.json" > "$OUT/pmc_args_summary.log" 2>&1 || true;; esac
case " $STEPS " in *" pmc "*) python tools/pmc_summary.py "$OUT/pmc" cgnni_bch_63_45_B65536_T25_f32 "$OUT/pmc_cgnni_bch_63_45_B65536_T25_f32.json" > "$OUT/pmc_summary.log" 2>&1 || true;; esac
echo "=== done $(date +%T)"
