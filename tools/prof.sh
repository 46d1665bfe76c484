# rocprofv3 kernel trace + PMC passes of one bench workload (profiles/collect.sh), summarised into
# gpurun_out/<tag>_<w> (copied to profiles/<tag>_<w> when committed). Usage: tools/prof.sh <tag> c2 c3 c4 c5 c2x
set -o pipefail
# one stderr line per launch attempt, so summarize.py can leave re-run launches out of the per-step count
export SIDDHI_HIP_DEBUG="SDH_TRACE=1"
tag=$1; shift
for w in $*; do
  case $w in
    c2) A="--steps 2 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency"; K=nfa_ratchet_kernel; P=10000; B=8388608;;
    c2x) A="--workload c2x --steps 2 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency"; K=${C2X_KERNEL:-nfa_gate_kernel}; P=10000; B=${C2X_BATCH:-4194304};;
    c3) A="--workload c3 --steps 4 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency"; K=sdh_part_spec; P=1000; B=1048576;;
    c4) A="--workload c4 --steps 4 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency"; K=sdh_seq_spec; P=10000; B=1048576;;
    c5) A="--workload c5 --no-cpu-baseline --no-calibrate"; K=nfa_slab_kernel; P=100000; B=524288;;
  esac
  [ "$w" = c2x ] && A="$A --batch $B"
  bash profiles/collect.sh gpurun_out/p_$w "$A" $K || exit 1
  python3 profiles/summarize.py gpurun_out/p_$w gpurun_out/${tag}_$w $K $w $P $B > gpurun_out/p_$w.sum || exit 1
  grep -E "kernel_ns|traffic|issue|bank" gpurun_out/p_$w.sum
  cp gpurun_out/p_$w/trace.log gpurun_out/${tag}_$w/trace.log
  rm -rf gpurun_out/p_$w  # (the raw per-dispatch CSVs: C5's exceed what a call copies back)
done
