#!/usr/bin/env bash
# One GPU session, parametrised: a sequence of steps, each under its own time
# limit, chained so that the first failure ends the session (no retries).
# Replaces the per-session gpu_r3*.sh scripts of round 3 (git history).
#
#   scripts/gpu_session.sh OUTDIR 'STEP ARGS...' ['STEP ARGS...' ...]
#
# Steps (outputs under OUTDIR, named by the step's index i):
#   tests [pytest args]         python -m pytest -m gpu (default: tests/)  -> i_pytest.log
#   smoke                       __graft_entry__.smoke()                   -> i_smoke.log
#   bench [bench.py args]       one bench line                            -> i_bench.json
#   kprof [bench.py args]       rocprofv3 --kernel-trace --stats of bench  -> i_prof/ + i_kernel_stats.txt
#   pmc COUNTERS SCRIPT [args]  one rocprofv3 --pmc pass of python3 SCRIPT args (counters
#                               comma-separated, one word)                 -> pmc/p<i>/
#   ab ROUNDS SPECFILE          interleaved A/B bench lines, one spec "label:ENV=..|bench args"
#                               per line of SPECFILE (scripts/ab/*.txt)   -> i_ab/
#   builders THREADS MODES R    tests/cpp/concurrent_builders, THREADS/MODES comma lists, R rounds
#                                                                          -> i_builders.jsonl
#   run SECONDS CMD...          any other command under its own limit      -> i_run.log
set -o pipefail
OUT=${1:?outdir}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i + 1))
  read -r kind rest <<< "$step"
  echo "[$(date +%H:%M:%S)] step $i: $kind $rest" >> "$OUT/session.log"
  case "$kind" in
    tests)
      timeout -k 10 900 python -u -m pytest ${rest:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/${i}_pytest.log" 2>&1 || { echo "step $i failed: $?" >> "$OUT/session.log"; exit 10; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${i}_smoke.log" 2>&1 ||
        { echo "step $i failed" >> "$OUT/session.log"; exit 11; } ;;
    bench)
      timeout -k 10 600 python -u bench.py $rest > "$OUT/${i}_bench.json" 2> "$OUT/${i}_bench.err" ||
        { echo "step $i failed" >> "$OUT/session.log"; exit 12; } ;;
    kprof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${i}_prof" -o run -- \
        python3 bench.py $rest > "$OUT/${i}_kprof.json" 2> "$OUT/${i}_kprof.err" ||
        { echo "step $i failed" >> "$OUT/session.log"; exit 13; }
      python3 scripts/kstats.py "$OUT/${i}_prof" > "$OUT/${i}_kernel_stats.txt" 2>&1 || true ;;
    pmc)
      # pmc COUNTERS SCRIPT [args]: one --pmc pass of `python3 SCRIPT args`
      read -r counters script brest <<< "$rest"
      timeout -s KILL 200 rocprofv3 --kernel-trace --pmc ${counters//,/ } --output-format csv -d "$OUT/pmc/p${i}" -o run -- \
        python3 $script $brest > "$OUT/${i}_pmc.json" 2> "$OUT/${i}_pmc.err" ||
        { echo "step $i failed" >> "$OUT/session.log"; exit 14; } ;;
    ab)
      # ab ROUNDS SPECFILE: one "label:ENV=..|bench args" spec per line of SPECFILE
      read -r rounds specfile <<< "$rest"
      mapfile -t specs < "$specfile"
      ROUNDS=$rounds timeout -k 10 1000 bash scripts/gpu_ab.sh "$OUT/${i}_ab" "${specs[@]}" ||
        { echo "step $i failed" >> "$OUT/session.log"; exit 15; } ;;
    builders)
      read -r threads modes rounds <<< "$rest"
      [ -x "$OUT/cb" ] || g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include \
        tests/cpp/concurrent_builders.cc -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle \
        -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib \
        -o "$OUT/cb" || { echo "step $i: build failed" >> "$OUT/session.log"; exit 16; }
      for r in $(seq 1 "${rounds:-3}"); do
        for mode in ${modes//,/ }; do
          for t in ${threads//,/ }; do
            timeout -k 10 180 "$OUT/cb" "$t" 8 153846 "$mode" >> "$OUT/${i}_builders.jsonl" 2>> "$OUT/${i}_builders.err" ||
              { echo "step $i failed ($mode $t)" >> "$OUT/session.log"; exit 17; }
          done
        done
      done ;;
    run)
      read -r secs cmd <<< "$rest"
      timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/${i}_run.log" 2>&1 ||
        { echo "step $i failed" >> "$OUT/session.log"; exit 18; } ;;
    *)
      echo "unknown step $kind" >> "$OUT/session.log"; exit 2 ;;
  esac
done
echo "[$(date +%H:%M:%S)] done" >> "$OUT/session.log"
