#!/bin/bash
# Counter evidence for what limits sqp_kernel (run on the GPU box via gpurun):
#   tools/pmc_latency.sh <round> <config> <batch>
# One rocprofv3 --pmc pass per counter group (each group within the gfx950
# per-pass slots: <= 8 SQ, <= 4 TCC with FETCH_SIZE = 3 and WRITE_SIZE = 2),
# each over one lone batch (bench.py --steps 1 --warmup 0 --inflight 1).
# tools/summarize_pmc.py then writes profiles/<round>_pmc_<config>.json.
set -e
ROUND=${1:-r03}
CFG=${2:-C}
BATCH=${3:-1024}
export TMPDIR=/tmp
D=gpurun_out/pmc_${CFG}
rm -rf "$D"
mkdir -p "$D"
BENCH="python3 bench.py --config $CFG --batch $BATCH --steps 1 --warmup 0 --inflight 1 --no-cpu"
pass() {
  local name=$1
  local extra=$2
  shift 2
  echo "pass $name: $*"
  timeout -s KILL 240 rocprofv3 $extra --pmc "$@" --output-format csv -d "$D/$name" -o p -- $BENCH > "$D/$name.log" 2>&1
}
pass waves --kernel-trace SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass issue "" SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_WAVE
pass insts "" SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH
pass lds "" SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F SQ_INSTS_VALU_ADD_F SQ_INSTS_VALU_MUL_F SQ_THREAD_CYCLES_VALU
pass fetch "" FETCH_SIZE
pass write "" WRITE_SIZE
python3 tools/summarize_pmc.py "$ROUND" "$CFG" "$BATCH"
