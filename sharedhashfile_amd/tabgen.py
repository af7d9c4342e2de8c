"""Synthetic tab images for the f4 tab part / shrink copy.

A tab image is the byte image of one reference tab file (SHF_TAB_MMAP,
/root/reference/src/shf.private.h:59-66): a 24-B header, 512 rows of 16
8-B refs {tab:11 | rnd:21, pos} (:48-56), then the key,value records its puts
appended (SHF_TAB_APPEND, /root/reference/src/shf.c:545-610): per record a
SHF_DATA_TYPE byte, u32 key length, key, u32 value length, value. The
reference parts a tab when the row a put needs is full (shf.c:829-834), so a
tab at part time holds a few thousand refs spread over its 512 rows, their
records in insertion order (not row order), and its refs' tab2 values are the
window entries that name the tab (the map redirect then sends every second one
to the new tab, shf.c:683-692).

Only the bench uses this (inputs for the tab-copy line); the tests use tab
files the reference itself wrote (tests/golden/tab_part_fixture.npz).
"""
import numpy as np

TAB_HDR = 24
TAB_REFS = 512 * 16
TAB_DATA = TAB_HDR + TAB_REFS * 8  # offsetof(SHF_TAB_MMAP, data)
PAGE = 4096


def mod_page(b):
    return ((b - 1) // PAGE + 1) * PAGE


def synth_tab(seed, n_refs=4500, key_lo=16, key_hi=64, val_lo=8, val_hi=128, owned_tab2=16, tab_old=7):
    """One variable-length store's tab at part time. Returns (image uint8,
    window map uint16[2048] before the redirect, tab_old)."""
    rng = np.random.default_rng(seed)
    slots = np.sort(rng.choice(TAB_REFS, n_refs, replace=False))  # ref index = row * 16 + ref
    owned = rng.choice(2048, owned_tab2, replace=False)
    tab2 = owned[rng.integers(0, owned_tab2, n_refs)].astype(np.uint32)
    rnd = rng.integers(0, 1 << 21, n_refs, dtype=np.uint32)
    kl = rng.integers(key_lo, key_hi + 1, n_refs)
    vl = rng.integers(val_lo, val_hi + 1, n_refs)
    rec = 1 + 4 + kl + 4 + vl
    order = rng.permutation(n_refs)  # insertion order of the records
    start = np.empty(n_refs, np.int64)
    start[order] = np.concatenate([[0], np.cumsum(rec[order])[:-1]])
    total = int(rec.sum())
    img = np.zeros(TAB_DATA + total, np.uint8)
    data = img[TAB_DATA:]
    payload = rng.integers(0, 256, total, dtype=np.uint8)  # key and value bytes
    for j in range(n_refs):
        s, k, v = int(start[j]), int(kl[j]), int(vl[j])
        data[s] = 0x3E  # SHF_DATA_TYPE: key and value STR32 (shf.private.h)
        data[s + 1:s + 5] = np.frombuffer(np.uint32(k).tobytes(), np.uint8)
        data[s + 5:s + 5 + k] = payload[s + 5:s + 5 + k]
        data[s + 5 + k:s + 9 + k] = np.frombuffer(np.uint32(v).tobytes(), np.uint8)
        data[s + 9 + k:s + 9 + k + v] = payload[s + 9 + k:s + 9 + k + v]
    rows = img[TAB_HDR:TAB_DATA].view(np.uint32).reshape(TAB_REFS, 2)
    rows[slots, 0] = tab2 | (rnd << np.uint32(11))
    rows[slots, 1] = (TAB_DATA + start).astype(np.uint32)
    hdr = img[:TAB_HDR].view(np.uint32)
    hdr[:] = [mod_page(TAB_DATA + total), TAB_DATA + total, 2 * n_refs, 0, 0, total]
    tab_map = rng.integers(0, 2048, 2048).astype(np.uint16)
    tab_map[tab_map == tab_old] = (tab_old + 1) % 2048
    tab_map[owned] = tab_old
    return img, tab_map, tab_old


def algorithmic_bytes(img, moving=True):
    """Bytes one part (moving) or shrink job reads and writes at least: the
    source header, rows and records once; each output's header and rows, and
    every record once more (its copy)."""
    data = int(img[:TAB_HDR].view(np.uint32)[5])
    return TAB_DATA + data + (2 if moving else 1) * TAB_DATA + data
