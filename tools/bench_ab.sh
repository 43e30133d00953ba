# Interleaved bench A/B on one GPU box: every variant once per round, ROUNDS rounds.
# usage: bash tools/bench_ab.sh TAG ROUNDS "BENCH ARGS" NAME:SETTING ...
#   SETTING = comma-separated VAR=VALUE pairs (e.g. DSR_PRESCAN=1,DSR_STREAMS=2), a library
#   (lib=dsp-slam-rgbd_amd/csrc/exp_X.so, run through DSR_LIB), or "-" for the defaults.
# Each run writes gpurun_out/TAG_NAME_ROUND.log (the bench JSON line last); the first GPU step
# that does not end normally stops the script.  Round 6 used it for the chunked-pass default
# (r6z, r6aa), the builds A/B (r6ad) and the 8-object pass windows (r6af).
# e.g. bash tools/bench_ab.sh r6af 2 "--objects 8 --steps 20 --warmup 3" default:- w20:DSR_TEST_HOOKS=1,DSR_RENDER_PASSES=20
set -u
mkdir -p gpurun_out
T=$1; R=$2; ARGS=$3; shift 3
for i in $(seq 1 $R); do
  for V in "$@"; do
    NAME=${V%%:*}; SET=${V#*:}
    ENVS=()
    if [ "$SET" != "-" ]; then
      IFS=',' read -ra KV <<< "$SET"
      for kv in "${KV[@]}"; do
        case $kv in
          lib=*) ENVS+=("DSR_LIB=$PWD/${kv#lib=}") ;;
          *) ENVS+=("$kv") ;;
        esac
      done
    fi
    env "${ENVS[@]}" timeout -k 10 300 python -u bench.py $ARGS --no-cpu-baseline --no-extra --no-config4 \
      > gpurun_out/${T}_${NAME}_$i.log 2>&1 || exit $?
  done
done
for f in gpurun_out/${T}_*.log; do
  echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"], 1), round(d["roofline"]["avg_launch_ms"], 4))')"
done
