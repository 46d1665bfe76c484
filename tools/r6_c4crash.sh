# Reproduce the round-5 lat_c4b core dump: C4 (unpartitioned K_seq) latency probe variants; stop at the first failure
set -o pipefail
run() {
  local name=$1; shift
  echo "cmd: python -X faulthandler -u tools/lat_probe.py $*" > gpurun_out/$name.log
  SDH_TRACE=1 timeout -k 10 120 python -X faulthandler -u tools/lat_probe.py "$@" >> gpurun_out/$name.log 2>&1
  local rc=$?
  echo "rc $rc" >> gpurun_out/$name.log
  echo "$name rc $rc"; tail -25 gpurun_out/$name.log
  return $rc
}
run c4x_compact --workload c4 --bs 1 --n 40 --compact && \
run c4x_reserve --workload c4 --bs 1 --n 40 --reserve && \
run c4x_both64 --workload c4 --bs 64 --n 40 --compact --reserve
