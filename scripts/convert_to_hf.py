#!/usr/bin/env python3
"""Same command line as the reference's ``scripts/convert_to_hf.py`` (``<checkpoint_path> [output_dir]
[--config_path ...] [--eos_token_id ...] [--dtype ...]``); runs ``llm-training convert-to-hf``
(llm_training_amd/tools/convert_to_hf.py), which reads this framework's checkpoints and the reference's
DeepSpeed / FSDP2 / Lightning ones."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llm_training_amd.cli.main import main  # noqa: E402

if __name__ == "__main__":
    # fire-style --key value / --key=value pass straight through to the argparse front end
    sys.exit(main(["convert-to-hf", *sys.argv[1:]]) or 0)
