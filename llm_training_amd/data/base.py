"""Data-module base classes and the resumable distributed sampler.

Reference: BaseDataModuleConfig (src/llm_training/data/base_datamodule_config.py:4-13), BaseDataModule
(data/base_datamodule.py: setup pipeline load -> pre_process -> post_process -> split :89-111, train
loader :71-87, dataset info :55-69) and ResumableDataLoader (data/resumable_dataloader.py:8-56).

Sharding is by DATA-parallel rank (TP ranks of one DP group see identical batches, reference
fsdp2_strategy.py:150-153). Resume is exact and cheap: the sampler's permutation is a function of
(seed, epoch) and skipping ``k`` batches slices the index list instead of iterating the loader.
"""
from __future__ import annotations

import logging
import math
from typing import Any, Iterator

import torch
from pydantic import BaseModel as PydanticModel
from pydantic import ConfigDict
from torch.utils.data import DataLoader, Dataset, Sampler

logger = logging.getLogger("llm_training")


class BaseDataModuleConfig(PydanticModel):
    model_config = ConfigDict(arbitrary_types_allowed=True, protected_namespaces=(), extra="forbid")

    pre_processed_data_path: str | None = None
    validation_split: int | float | None = None
    batch_size: int = 1
    num_workers: int = 0
    pin_memory: bool = False
    prepare_data_per_node: bool = False
    prefetch_factor: int | None = None


class ResumableDistributedSampler(Sampler[list[int]]):
    """Batch sampler: seeded per-epoch permutation, DP-rank strided, skip-k-batches resume."""

    def __init__(self, n: int, batch_size: int, dp_rank: int = 0, dp_size: int = 1, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = True):
        self.n, self.bs, self.rank, self.world = n, batch_size, dp_rank, dp_size
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        self.skip = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def set_skip(self, batches: int):
        self.skip = int(batches)

    def _indices(self) -> list[int]:
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        per = self.n // self.world if self.drop_last else math.ceil(self.n / self.world)
        if not self.drop_last and per * self.world > self.n:
            idx = idx + idx[: per * self.world - self.n]
        return idx[self.rank: per * self.world: self.world]

    def __iter__(self) -> Iterator[list[int]]:
        idx = self._indices()
        nb = len(self)
        for b in range(self.skip, nb):
            yield idx[b * self.bs:(b + 1) * self.bs]
        self.skip = 0

    def __len__(self) -> int:
        per = self.n // self.world if self.drop_last else math.ceil(self.n / self.world)
        return per // self.bs if self.drop_last else math.ceil(per / self.bs)


def default_collate(items: list[dict]) -> dict:
    out: dict[str, Any] = {}
    for k in items[0]:
        v = [it[k] for it in items]
        out[k] = torch.stack([torch.as_tensor(x) for x in v]) if isinstance(v[0], (torch.Tensor, list)) else v
    if "attention_mask" in out and isinstance(out["attention_mask"], torch.Tensor):
        out["attention_mask_trivial"] = bool((out["attention_mask"] == 1).all())
    return out


class BaseDataModule:
    config_class = BaseDataModuleConfig

    def __init__(self, config: BaseDataModuleConfig | dict):
        if isinstance(config, dict):
            config = self.config_class.model_validate(config)
        self.config = config
        self.datasets: dict[str, Dataset] = {}
        self.collator = self.build_collator()

    def build_collator(self):
        return default_collate

    # pipeline (override pieces)
    def prepare_data(self):
        pass

    def load_data(self):
        raise NotImplementedError

    def pre_process_data(self, datasets):
        return datasets

    def post_process_data(self, datasets):
        return datasets

    def setup(self, stage: str | None = None):
        if self.config.pre_processed_data_path:
            ds = self.load_pre_processed_data(self.config.pre_processed_data_path)
        else:
            ds = self.pre_process_data(self.load_data())
        self.pre_processed_datasets = ds
        self.datasets = self.post_process_data(self.split(ds))

    def split(self, ds):
        if isinstance(ds, dict):
            return ds
        vs = self.config.validation_split
        if not vs:
            return {"train": ds}
        n = len(ds)
        nv = int(vs if isinstance(vs, int) and not isinstance(vs, bool) and vs >= 1 else round(n * float(vs)))
        g = torch.Generator().manual_seed(42)
        perm = torch.randperm(n, generator=g).tolist()
        return {"train": _Subset(ds, perm[nv:]), "validation": _Subset(ds, perm[:nv])}

    def load_pre_processed_data(self, path):
        import datasets as hfd
        return hfd.load_from_disk(path)

    def save_pre_processed_data(self, path):
        for k, d in self.datasets.items():
            d.save_to_disk(f"{path}/{k}")

    def train_dataloader(self, dp_rank=0, dp_size=1, seed=0, skip_batches=0, epoch=0, shuffle=True) -> DataLoader:
        ds = self.datasets["train"]
        sampler = ResumableDistributedSampler(len(ds), self.config.batch_size, dp_rank, dp_size, shuffle, seed)
        sampler.set_epoch(epoch)
        sampler.set_skip(skip_batches)
        kw = {}
        if self.config.num_workers > 0 and self.config.prefetch_factor:
            kw["prefetch_factor"] = self.config.prefetch_factor
        # a loader-owned generator for the worker base seed: creating the iterator (again after a resume)
        # must not draw from the global generator that dropout / NEFTune consume
        gen = torch.Generator().manual_seed(seed * 1_000_003 + epoch * 7919 + dp_rank)
        return DataLoader(ds, batch_sampler=sampler, collate_fn=self.collator, num_workers=self.config.num_workers,
                          pin_memory=self.config.pin_memory, persistent_workers=False, generator=gen, **kw)

    def val_dataloader(self, dp_rank=0, dp_size=1) -> DataLoader | None:
        ds = self.datasets.get("validation")
        if ds is None:
            return None
        sampler = ResumableDistributedSampler(len(ds), self.config.batch_size, dp_rank, dp_size, False, 0,
                                              drop_last=False)
        return DataLoader(ds, batch_sampler=sampler, collate_fn=self.collator, num_workers=self.config.num_workers,
                          generator=torch.Generator().manual_seed(dp_rank))

    def print_dataset_info(self):
        for k, d in self.datasets.items():
            logger.info("dataset %s: %d examples", k, len(d))


class _Subset(Dataset):
    def __init__(self, ds, idx):
        self.ds, self.idx = ds, idx

    def __len__(self):
        return len(self.idx)

    def __getitem__(self, i):
        return self.ds[self.idx[i]]
