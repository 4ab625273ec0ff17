#!/usr/bin/env bash
# SLURM launcher for multi-node MI355X training: one task per GPU (srun), RCCL over xGMI inside a
# node and RoCE/IB between nodes. Ranks, MASTER_ADDR/PORT come from the SLURM environment
# (llm_training_amd/parallel/context.py). Mirrors the reference's scripts/train.sh interface.
#
#   CONFIG=config/examples/llama-3/llama-3-8b_pt_mi355x.yaml NODES=2 PARTITION=mi355x scripts/train.sh
set -euo pipefail

JOB_NAME=${JOB_NAME:-llm-training}
PARTITION=${PARTITION:-}
ACCOUNT=${ACCOUNT:-}
NODES=${NODES:-1}
GPUS_PER_NODE=${GPUS_PER_NODE:-8}
CPUS_PER_TASK=${CPUS_PER_TASK:-16}
CONFIG=${CONFIG:?set CONFIG=<yaml>}
CKPT_PATH=${CKPT_PATH:-null}
EXTRA_ARGS=(${EXTRA_ARGS:-})

# dmabuf IPC (legacy IPC handles are not supported by the MI355X host driver)
export HSA_ENABLE_IPC_MODE_LEGACY=0
# one RCCL channel set per xGMI link; NCCL_* names are honoured by RCCL
export NCCL_MIN_NCHANNELS=${NCCL_MIN_NCHANNELS:-16}
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-8}

COMMAND="srun --cpu-bind=none llm-training fit --config $CONFIG --trainer.num_nodes $NODES --ckpt_path $CKPT_PATH"
echo "$COMMAND"

SBATCH_ARGS=(--job-name "$JOB_NAME" --nodes "$NODES" --gpus-per-node "$GPUS_PER_NODE"
             --ntasks-per-node "$GPUS_PER_NODE" --cpus-per-task "$CPUS_PER_TASK")
[[ -n "$PARTITION" ]] && SBATCH_ARGS+=(--partition "$PARTITION")
[[ -n "$ACCOUNT" ]] && SBATCH_ARGS+=(--account "$ACCOUNT")
SBATCH_ARGS+=("${EXTRA_ARGS[@]}")

OUT=$(sbatch "${SBATCH_ARGS[@]}" --wrap "$COMMAND")
echo "$OUT"
[[ "$OUT" == "Submitted batch job"* ]] || exit 1
JOB_ID=${OUT#Submitted batch job }

echo "waiting for job $JOB_ID to start"
until [[ "$(squeue -j "$JOB_ID" -h -o %T)" == "RUNNING" ]]; do sleep 2; done
sleep 3
# follow step 0's output until it ends
sattach "$JOB_ID.0" || true
