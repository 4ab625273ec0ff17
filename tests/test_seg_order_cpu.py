"""Packed-row block orders of ops/fused.py segment_info (the flash kernels' a.qord / a.kord) and the per-problem
stream-K twins of the GEMM layout candidates (_sk_pairs), on the CPU."""
import pytest
import torch

from llm_training_amd.ops import fused as F_


def _rows(B, S, docs, seed):
    g = torch.Generator().manual_seed(seed)
    seg = torch.empty(B, S, dtype=torch.int32)
    for b in range(B):
        cuts = sorted(torch.randperm(S - 1, generator=g)[: docs - 1].add(1).tolist())
        e = [0, *cuts, S]
        seg[b] = torch.repeat_interleave(torch.arange(1, docs + 1, dtype=torch.int32),
                                         torch.tensor([y - x for x, y in zip(e[:-1], e[1:])]))
    return seg


def _orders(info, B, S):
    nb = (S + 127) // 128
    q = info[3 * B * S: 3 * B * S + B * nb].long()
    k = info[3 * B * S + B * nb:].long()
    return q, k, nb


@pytest.mark.parametrize("docs", [1, 3, 8, 32])
def test_doc_major_order_is_a_permutation_grouped_by_document(docs, monkeypatch):
    monkeypatch.delenv("LLMT_SEG_ORDER", raising=False)
    B, S = 3, 2048
    seg = _rows(B, S, docs, docs)
    info = F_.segment_info(seg, doc_major=True)
    q, k, nb = _orders(info, B, S)
    runs = info[: 3 * B * S].view(3, B, S)
    rs, re = runs[1].long(), runs[2].long()
    for order, work in ((q, "q"), (k, "k")):
        assert sorted(order.tolist()) == list(range(B * nb))  # every (row, block) exactly once
        # the document of a block = the run of its last token; each document's blocks are one contiguous run
        # of the order, and documents come longest first
        docs_seen, last, lens = [], None, []
        for bm in order.tolist():
            b, blk = divmod(bm, nb)
            t = min(blk * 128 + 127, S - 1)
            d = (b, int(rs[b, t]))
            if d != last:
                assert d not in docs_seen, "a document's blocks are split"
                docs_seen.append(d)
                lens.append(int(re[b, t]) - int(rs[b, t]) + 1)
                last = d
        assert lens == sorted(lens, reverse=True)


def test_doc_major_heaviest_block_first_inside_a_document(monkeypatch):
    monkeypatch.delenv("LLMT_SEG_ORDER", raising=False)
    B, S = 1, 4096
    seg = (torch.arange(S) * 2 // S + 1).to(torch.int32).view(1, S)  # two 2048-token documents
    q, k, nb = _orders(F_.segment_info(seg, doc_major=True), B, S)
    # query blocks: the later a block sits in its document, the more key tiles it has (causal)
    assert q[:16].tolist() == list(range(15, -1, -1)) or q[:16].tolist() == list(range(31, 15, -1))
    # key blocks: the earlier, the more query tiles
    assert k[:16].tolist() in (list(range(16)), list(range(16, 32)))


def test_default_order_is_heaviest_first_and_env_overrides(monkeypatch):
    monkeypatch.delenv("LLMT_SEG_ORDER", raising=False)
    B, S = 2, 1024
    seg = _rows(B, S, 4, 7)
    a = F_.segment_info(seg)
    monkeypatch.setenv("LLMT_SEG_ORDER", "1")
    assert torch.equal(a, F_.segment_info(seg, doc_major=True))  # the environment pins the order
    monkeypatch.setenv("LLMT_SEG_ORDER", "0")
    assert F_.segment_info(seg).numel() == 3 * B * S  # index order: the run layout alone
    monkeypatch.setenv("LLMT_SEG_ORDER", "2")
    assert not torch.equal(a, F_.segment_info(seg))


@pytest.mark.parametrize("allowed", [True, False])
def test_sk_pairs_twin_every_layout_with_stream_k(allowed, monkeypatch):
    monkeypatch.setattr(F_, "ALLOW_STREAMK", [allowed])
    calls = []
    v = F_._sk_pairs({"tn": lambda s: calls.append(("tn", s)), "nn": lambda s: calls.append(("nn", s))})
    if allowed:
        assert sorted(v) == ["nn", "nn/nosk", "tn", "tn/nosk"]
    else:
        assert sorted(v) == ["nn", "tn"]
    for name in sorted(v):
        v[name]()
    want = [("nn", allowed), ("nn", False), ("tn", allowed), ("tn", False)] if allowed else [("nn", False), ("tn", False)]
    assert calls == want
