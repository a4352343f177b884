#!/bin/bash
# Round-4 session h on the shipped build: recovery tests + same-box A/B of the
# partial decode with inlined membership (head vs libdrand_gpu_conf.so), then
# the rocprofv3 kernel-trace statistics of the headline bench command and the
# PMC passes (VALU / LDS / occupancy counters, HBM traffic) of the per-round
# pipeline -- one rocprofv3 run per pass, kernel trace only.
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/${HTAG:-r04h}
mkdir -p $O
if [ -z "$NOAB" ]; then
TAG=r04h1 PYTEST_K="recover" REPS=1 VARIANTS="head=X conf=LIB=libdrand_gpu_conf.so" BENCH_ARGS="--mode recover --steps 3 --no-cpu-baseline" bash tools/gpu/r04_ab.sh || exit $?
fi
if [ -z "$NOPROF" ]; then
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --no-legs --steps 2 > $O/prof.out 2>&1 || exit $?
python3 tools/rocpd_stats.py $(find $O/prof -name "*results.db" | head -1) > $O/kernel_stats.csv || true
ls $O/prof
fi
if [ -z "$NOPMC" ]; then
P=$O/pmc
mkdir -p $P
run() {  # name, counters
  step "pmc $1"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d $P/$1 -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > $P/$1.log 2>&1
}
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" || exit $?
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" || exit $?
run sq3 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" || exit $?
run fetch "FETCH_SIZE" || exit $?
run write "WRITE_SIZE" || exit $?
python3 tools/pmc_summary.py $P > $P/pmc_summary.txt
python3 tools/traffic_summary.py $P 131072 $P/traffic.json > $P/traffic.log
fi
echo done
