# v18b: VALU utilisation PMC pass (raw counters for VALUBusy / VALUUtilization)
# and the dLSM-realistic 153,846-key SSTable variant of the bench.
set -o pipefail
O=gpurun_out/v18b
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d $O/valu -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > $O/valu.json 2> $O/valu.err &&
timeout -k 10 300 python bench.py --keys-per-table 153846 --no-e2e --steps 50 --warmup 10 > $O/n153846.json 2> $O/n153846.err
