set -e
O=gpurun_out/r5d
mkdir -p $O
for ps in 1024 256 64; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$ps -o run -- python3 scripts/bench_version_probe.py --lookups 100000000 --reps 2 --check 0 --paths sliced --slice-bytes 20000000 --pass-slices $ps > $O/p$ps.json 2> $O/p$ps.err
done
python3 scripts/shrink_outputs.py $O
