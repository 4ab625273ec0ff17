#!/usr/bin/env python3
"""Same command line as the reference's ``scripts/pre_process_data.py`` (``-c/--config <yaml>`` plus
overrides): tokenizes / packs the data module's dataset once and saves it to
``data.init_args.config.pre_processed_data_path`` (``llm-training pre-process``)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llm_training_amd.cli.main import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["pre-process", *sys.argv[1:]]) or 0)
