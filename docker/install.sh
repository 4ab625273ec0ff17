#!/usr/bin/env bash
# Build the gfx950 HIP extension in-tree and install the package (editable, `llm-training` on PATH).
# Reference: install.sh (flash-attn build + pip install -e .[deepspeed]).
set -euo pipefail
cd "$(dirname "$0")/.."
export LLMT_OFFLOAD_ARCH=${LLMT_OFFLOAD_ARCH:-gfx950}
python -m llm_training_amd._build
pip install --no-build-isolation --no-deps -e .
python -c "import llm_training_amd.ops.native as n; assert n.available(), n._ERR; print('native extension ok')"
