#!/bin/bash
# Round-4 session p: RLC bucket-run length A/B (k_msm_window: 64 buckets per
# thread, the default, vs 16 / 8: more threads, shorter serial runs, two or
# three more pairwise levels), chained 10M RLC at 0.1% corrupted and on-G1
# RLC 10M; then the RLC GPU tests on the 8-bucket build.
export TMPDIR=/tmp
TAG=r04p1 REPS=2 VARIANTS="r64=X r16=LIB=libdrand_gpu_r16.so r8=LIB=libdrand_gpu_r8.so" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
TAG=r04p2 REPS=1 VARIANTS="r64=X r8=LIB=libdrand_gpu_r8.so" BENCH_ARGS="--mode rlc --scheme bls-unchained-on-g1 --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
# PMC of the RLC pipeline's kernels (k_msm_bucket, k_rlc_prep, ...) at 2M rounds
P=gpurun_out/r04p/pmc
mkdir -p $P
run() {  # name, counters
  echo "== pmc $1 $(date +%T)"
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d $P/$1 -o p -- python3 bench.py --mode rlc --rounds 2000000 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-legs > $P/$1.log 2>&1
}
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" || exit $?
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" || exit $?
run fetch "FETCH_SIZE" || exit $?
python3 tools/pmc_summary.py $P > $P/pmc_summary.txt
echo done
