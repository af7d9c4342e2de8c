"""Synthetic row indexes for the row pre-probe.

A real index is exported from a live store (the tests use
the reference's own store through oracle/ref_export.c). For benchmarks at
BASELINE sizes, and for parity cases the reference store cannot produce
(ragged slots, dangling tab_slot entries), this module lays out an index in
the same format (include/shf_hash_batch.h) from a batch of hashes:

  * every window has `tabs_per_win` physical tabs; tab2 maps to tab
    tab2 % tabs_per_win (a valid SHF_WIN_MMAP.tabs[] state, cf. the initial
    round-robin map at /root/reference/src/shf.c:425-433);
  * slot = win * tabs_per_win + tab;
  * each key takes the next free ref of its row, in batch order, with
    pos = key index + 1 (pos 0 means unused, shf.private.h:51); refs past 16
    per row are dropped (the reference would part the tab instead).

It is a data generator, not the reference's put: placement within a row
follows batch order, as put's first-free-ref scan does (shf.c:809-827) when
nothing was ever deleted.

Works on numpy arrays (CPU) or torch tensors (any device) with the same code.
"""
import numpy as np

REFS_PER_ROW = 16
ROWS_PER_TAB = 512
TABS = 256 * 2048
NONE = 0xFFFFFFFF


def _parts(h1, h2):
    win = h1 & 0xFF
    tab2 = (h1 >> 16) & 0x7FF
    row = (h1 >> 32) & 0x1FF
    rnd = h2 & 0x1FFFFF
    return win, tab2, row, rnd


def synthetic_index(hashes, tabs_per_win=1, limit=None):
    """(tab_slot u32[256*2048], rows u8[n_slots*65536], n_slots, placed) for `hashes` (n, 2).

    hashes: numpy uint64 / torch int64 (bit patterns) array of SHF_HASH records.
    limit: put only the first `limit` keys (the rest stay absent).
    """
    try:
        import torch

        is_torch = isinstance(hashes, torch.Tensor)
    except ImportError:  # pragma: no cover
        is_torch = False
    T = int(tabs_per_win)
    assert 1 <= T <= 2048
    n_slots = 256 * T
    n = hashes.shape[0] if limit is None else min(int(limit), hashes.shape[0])
    if is_torch:
        import torch

        dev = hashes.device
        h = hashes[:n].to(torch.int64)
        h1, h2 = h[:, 0], h[:, 1]
        win, tab2, row, rnd = _parts(h1, h2)
        w = torch.arange(256, device=dev, dtype=torch.int64).repeat_interleave(2048)
        t2 = torch.arange(2048, device=dev, dtype=torch.int64).repeat(256)
        tab_slot = ((w * T + t2 % T) << 11) | (t2 % T)
        slot = win * T + tab2 % T
        rid = slot * ROWS_PER_TAB + row
        order = torch.sort(rid, stable=True).indices
        rs = rid[order]
        idx = torch.arange(n, device=dev, dtype=torch.int64)
        first = torch.ones(n, dtype=torch.bool, device=dev)
        if n > 1:
            first[1:] = rs[1:] != rs[:-1]
        start = torch.cummax(torch.where(first, idx, torch.zeros_like(idx)), dim=0).values
        rank = idx - start
        keep = rank < REFS_PER_ROW
        ko = order[keep]
        ref = rid[ko] * REFS_PER_ROW + rank[keep]
        words = torch.zeros(n_slots * ROWS_PER_TAB * REFS_PER_ROW * 2, dtype=torch.int32, device=dev)
        word = (tab2[ko] | (rnd[ko] << 11)).to(torch.int64)
        word = torch.where(word >= 2**31, word - 2**32, word).to(torch.int32)
        words[ref * 2] = word
        words[ref * 2 + 1] = (ko + 1).to(torch.int32)
        tab_slot = torch.where(tab_slot >= 2**31, tab_slot - 2**32, tab_slot).to(torch.int32)
        return tab_slot, words.view(torch.uint8), n_slots, int(keep.sum())
    h = np.ascontiguousarray(hashes[:n], dtype=np.uint64)
    win, tab2, row, rnd = _parts(h[:, 0], h[:, 1])
    w = np.repeat(np.arange(256, dtype=np.uint64), 2048)
    t2 = np.tile(np.arange(2048, dtype=np.uint64), 256)
    tab_slot = (((w * T + t2 % T) << np.uint64(11)) | (t2 % T)).astype(np.uint32)
    slot = win * np.uint64(T) + tab2 % np.uint64(T)
    rid = (slot * np.uint64(ROWS_PER_TAB) + row).astype(np.int64)
    order = np.argsort(rid, kind="stable")
    rs = rid[order]
    idx = np.arange(n, dtype=np.int64)
    first = np.ones(n, dtype=bool)
    first[1:] = rs[1:] != rs[:-1]
    start = np.maximum.accumulate(np.where(first, idx, 0)) if n else idx
    rank = idx - start
    keep = rank < REFS_PER_ROW
    ko = order[keep]
    ref = rid[ko] * REFS_PER_ROW + rank[keep]
    words = np.zeros(n_slots * ROWS_PER_TAB * REFS_PER_ROW * 2, dtype=np.uint32)
    words[ref * 2] = (tab2[ko] | (rnd[ko] << np.uint64(11))).astype(np.uint32)
    words[ref * 2 + 1] = (ko + 1).astype(np.uint32)
    return tab_slot, words.view(np.uint8), n_slots, int(keep.sum())
