"""Data-only entry (reference scripts/pre_process_data.py:25-47): build the datamodule from
the YAML config, run its pipeline, save the processed datasets and an ``info.txt`` with token tables."""
from __future__ import annotations

import io
import logging
import os
from contextlib import redirect_stdout

logger = logging.getLogger("llm_training")


def pre_process(configs: list[str], overrides: list[str] | None = None):
    from ..config.loader import instantiate, load_config

    cfg = load_config(configs, overrides)
    dm = instantiate(cfg["data"])
    path = dm.config.pre_processed_data_path
    if not path:
        raise ValueError("data.init_args.config.pre_processed_data_path must be set")
    if os.path.isdir(path) and os.listdir(path):
        # as the reference: an existing non-empty output is kept (loaded, only info.txt is rewritten)
        logger.info("pre_processed_data_path=%s is not empty, skipping", path)
        dm.setup()
    else:
        dm.config.pre_processed_data_path = None
        dm.prepare_data()
        dm.setup()
        dm.save_pre_processed_data(path)
    buf = io.StringIO()
    with redirect_stdout(buf):
        dm.print_dataset_info()
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "info.txt"), "w") as f:
        f.write(buf.getvalue())
    logger.info("pre-processed data saved to %s", path)
    return path
