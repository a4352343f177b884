#!/bin/bash
# One parameterised GPU session (replaces the per-session r0*_*.sh scripts of
# rounds 2-4, which are in git history).  Usage, from the repo root:
#
#   TAG=r05a bash tools/gpu/session.sh STEP [STEP ...]
#
# Steps run in order; the first failure (or time limit) ends the session, so
# nothing else touches the GPU after a fault.  Output: gpurun_out/$TAG/.
#   pytest     GPU suite (PYTEST_SEL: test files / -k expression; default tests -m gpu)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py $BENCH_ARGS  -> bench.json (default: every leg)
#   prof       rocprofv3 --kernel-trace --stats of the headline command -> kernel_stats.csv
#   traffic    FETCH_SIZE / WRITE_SIZE passes of tools/prof_verify.py -> traffic.json
#              (TRAFFIC_ARGS: prof_verify options, default one 131072-round chunk)
#   pmc        the SQ/TCC counter passes of tools/pmc.sh over prof_verify -> pmc/
#   ab         bench each library in $VARIANTS (DRAND_GPU_LIB) with $BENCH_ARGS -> ab/<name>.json
#   small      the small-batch latency curve (bench.py --small-batch-only) -> small.json
#   abi8       the 8-GPU host side rehearsed on one GPU: dgpu_verify_multi over 8
#              loopback contexts of device 0 (10M rounds, 1.25M per shard), with
#              each shard's staging time through its context's pinned ring -> abi8.json
export TMPDIR=/tmp
TAG=${TAG:-session}
O=gpurun_out/$TAG
mkdir -p $O
say() { echo "== $1 $(date +%T)"; }
run_step() {
  case "$1" in
  pytest)
    timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests} -v -m gpu --timeout 240 --timeout-method thread \
      > $O/pytest.log 2>&1
    rc=$?; tail -3 $O/pytest.log; return $rc ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
    rc=$?; tail -1 $O/smoke.log; return $rc ;;
  bench)
    timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err
    rc=$?; head -c 400 $O/bench.json; echo; return $rc ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- \
      python3 bench.py --no-cpu-baseline --no-e2e --no-legs --steps 2 ${PROF_ARGS} > $O/prof.out 2>&1 || return $?
    python3 tools/rocpd_stats.py $(find $O/prof -name "*results.db" | head -1) > $O/kernel_stats.csv || true ;;
  traffic)
    # the third pass runs the engine lines kernel, whose 45,696 B/round of
    # stores calibrate WRITE_SIZE (tools/traffic_summary.py)
    for pass in fetch:FETCH_SIZE write:WRITE_SIZE write_cal:WRITE_SIZE; do
      name=${pass%%:*}
      ( [ $name = write_cal ] && export DGPU_LINES=engine
        timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc ${pass#*:} -d $O/traffic/$name -o p \
          -- python3 tools/prof_verify.py ${TRAFFIC_ARGS:---rounds 131072 --iters 1} > $O/traffic_$name.log 2>&1 ) \
        || return $?
    done
    python3 tools/traffic_summary.py $O/traffic ${TRAFFIC_ROUNDS:-131072} $O/traffic.json ;;
  pmc)
    TAG=$TAG/pmc PROF_ARGS="${TRAFFIC_ARGS:---rounds 131072 --iters 1}" bash tools/gpu/pmc.sh > $O/pmc.log 2>&1 ;;
  ab)
    mkdir -p $O/ab
    # a variant is lib.so or lib.so@KEY=VALUE[@KEY=VALUE...] (environment knobs read at dgpu_open)
    for v in $VARIANTS; do
      lib=${v%%@*}; kvs=$([ "$lib" != "$v" ] && echo "${v#*@}" | tr '@' ' ')
      name=$(basename $lib .so)$(for kv in $kvs; do echo -n "_${kv//=/_}"; done)
      ( for kv in $kvs; do export "$kv"; done
        DRAND_GPU_LIB=$PWD/$lib timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} \
          > $O/ab/ab_$name.json 2> $O/ab/ab_$name.err ) || return $?
    done
    python3 tools/ab_summary.py $O/ab ;;
  small)
    timeout -k 10 600 python -u bench.py --small-batch-only > $O/small.json 2> $O/small.err
    rc=$?; cat $O/small.json; return $rc ;;
  abi8)
    DGPU_MULTI_ALLOW_SAME_DEVICE=1 DGPU_ENG_CHUNK=131072 timeout -k 10 600 python -u bench.py --driver abi --gpus 8 \
      --abi-devices 0,0,0,0,0,0,0,0 --steps ${ABI8_STEPS:-2} --warmup 1 > $O/abi8.json 2> $O/abi8.err
    rc=$?; head -c 600 $O/abi8.json; echo; return $rc ;;
  *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  say $s
  run_step $s || { rc=$?; echo "step $s failed ($rc)"; exit $rc; }
done
echo done
