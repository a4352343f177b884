#!/bin/bash
# Round-4 session y: RLC-mode batches under DGPU_RLC_MIN (131,072 rounds) on
# the per-round path: GPU suite (the suite itself sets DGPU_RLC_MIN=0 so its
# small RLC batches take the RLC path; one test checks the default), smoke,
# then the throughput-against-batch-size curve again.
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for n in 4096 65536 131072 524288 2097152; do
  echo "== n=$n $(date +%T)"
  timeout -k 10 300 python -u bench.py --rounds $n --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-legs > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
echo done
