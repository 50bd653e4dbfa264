# Run GPU steps in order, each under its own time limit; a step that ends with a fault, an abort,
# a segfault or a timeout (any status other than 0 / 1) stops the sequence.
# usage: bash tools/gpu_seq.sh "<limit_s> <logname> <command...>" ...
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out/seq
export TMPDIR=/tmp
for step in "$@"; do
  lim=${step%% *}; rest=${step#* }; name=${rest%% *}; cmd=${rest#* }
  echo "== $name: $cmd"
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/seq/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/seq/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
