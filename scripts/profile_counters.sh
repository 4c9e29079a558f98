#!/bin/bash
# rocprofv3 hardware-counter passes over the flagship bench:
# MFMA work/busy, LDS bank conflicts, HBM traffic per HIP kernel. Counter runs
# use only --pmc (+ kernel trace), never a sys/runtime trace.
#   bash scripts/profile_counters.sh            (on the GPU box; outputs gpurun_out/pmc/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/${PMC_OUT:-pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 60 --warmup 10"}
i=0
# (pass 1: MFMA ops of every type the builds use -- bf16 (_C), fp16 (_C_f16: Rainbow), fp32 (_C_f32) --
#  6 SQ + 1 GRBM counters, within one pass's 8 SQ / 2 GRBM)
for group in "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
             "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace -d "$OUT/pass$i" -o pass$i --output-format csv -- \
      python3 "$REPO/bench.py" $ARGS > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "[pmc pass $i: $group] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
python3 "$REPO/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.md" && cat "$OUT/summary.md"
