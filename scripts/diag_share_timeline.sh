set -e
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5n/share8_trace -o run -- python3 bench.py --native --tables 2 --lookups 12500000 --steps 40 --warmup 5 --no-cpu --no-e2e --no-legacy --no-version --no-mixed > gpurun_out/r5n/share8_trace.json
python3 scripts/timeline.py gpurun_out/r5n/share8_trace --steps 30
