"""f4 on the GPU: the device tab part / shrink copy (shf_tab_copy_batch*,
include/shf_hash_batch.h) against the tab files the reference itself wrote
(tests/golden/tab_part_fixture.npz and live captures from oracle/_ref) and
against the CPU oracle (oracle/tab_oracle.c), bit-exact: header, all 512
rows, the data.
"""
import ctypes

import numpy as np
import pytest

import tabcheck
from oracle.oracle_py import reference_lib
from test_tab_oracle import fixture_caps

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(hb):
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    hb.check_device()
    return torch.device("cuda:0")


def gpu_part(hb, cap):
    m = hb.tab_part_redirect(cap["map_before"], cap["tab_old"], cap["tab_new"])
    kt, mt = tabcheck.observed_types(cap)
    params = dict(fixed=cap["fixed"], key_len=cap["fixed_key_len"], val_len=cap["fixed_val_len"],
                  factor=cap["factor"])
    return m, hb.tab_copy([cap["before"]], [m], [cap["tab_new"]], keep_type=kt, move_type=mt, **params)[0]


@pytest.mark.parametrize("i", [0, 1])
def test_part_matches_reference_fixture(hb, dev, i):
    cap = fixture_caps()[i]
    m, (keep, move) = gpu_part(hb, cap)
    assert np.array_equal(m, cap["map_after"])
    tabcheck.check_capture(cap, keep, move, cap["put_key_len"])


@pytest.mark.skipif(reference_lib() is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("lo,hi,fk,fv,fac", [(8, 40, 0, 0, 1), (16, 16, 16, 8, 3), (8, 200, 0, 0, 2),
                                            (32, 32, 32, 100, 1)])
def test_part_matches_live_reference(hb, dev, oracle, lo, hi, fk, fv, fac):
    from golden.make_tab_golden import window0_keys
    from oracle.oracle_py import reference_part_capture

    data, off = window0_keys(oracle, 3_000_000, lo, hi, 91 + lo + fv)
    caps = reference_part_capture(data, off, fixed_key_len=fk, fixed_val_len=fv, factor=fac, max_caps=3)
    assert len(caps) >= 2
    for cap in caps:
        _, (keep, move) = gpu_part(hb, cap)
        tabcheck.check_capture(cap, keep, move, int(off[cap["key"] + 1] - off[cap["key"]]))


def test_batch_of_parts_and_shrinks_matches_oracle(hb, dev, oracle):
    """64 jobs in one launch: parts to every other tab number and shrinks,
    over the fixture's tabs with maps that move different tab2 subsets."""
    caps = fixture_caps()
    rng = np.random.default_rng(5)
    images, maps, news, params = [], [], [], []
    for i in range(64):
        cap = caps[i % 2]
        m = np.array(cap["map_before"], dtype=np.uint16)
        if i % 3 == 2:
            news.append(hb.TAB_NONE)  # shrink only
        else:
            new = int(rng.integers(1, 2048))
            m[rng.random(2048) < 0.5] = new  # an arbitrary subset of tab2s moves
            news.append(new)
        images.append(cap["before"])
        maps.append(m)
    # one launch per store kind (the params are per launch)
    for kind in (0, 1):
        idx = [i for i in range(64) if i % 2 == kind]
        cap = caps[kind]
        kw = dict(fixed=cap["fixed"], key_len=cap["fixed_key_len"], val_len=cap["fixed_val_len"], factor=cap["factor"])
        got = hb.tab_copy([images[i] for i in idx], [maps[i] for i in idx], [news[i] for i in idx],
                          keep_type=0x3E, move_type=0xBE, **kw)
        for (keep, move), i in zip(got, idx):
            wk, wm = oracle.tab_split(images[i], maps[i], news[i], kw["fixed"], kw["key_len"], kw["val_len"],
                                      kw["factor"], cap=keep.size, keep_type=0x3E, move_type=0xBE)
            assert np.array_equal(keep, wk), i
            if news[i] == hb.TAB_NONE:
                assert move is None
            else:
                assert np.array_equal(move, wm), i


def test_shrink_of_a_shrunk_tab_is_the_same_tab(hb, dev):
    cap = fixture_caps()[0]
    keep, _ = hb.tab_copy([cap["before"]], None, None)[0]
    again, _ = hb.tab_copy([keep[:tabcheck.hdr(keep)[0]]], None, None)[0]
    assert np.array_equal(again[:keep.size], keep)


def test_malformed_jobs_fail_without_fault(hb, dev):
    """Jobs naming bytes outside their buffers, outputs too small, a ref whose
    record runs past the image, misaligned images: status ERR_ARG, no fault,
    and the good job of the same launch still done."""
    lib = hb.load()
    cap = fixture_caps()[0]
    img = np.array(cap["before"], dtype=np.uint8)
    corrupt = img.copy()
    rows = corrupt[24:65560].view(np.uint32).reshape(-1, 2)
    first = int(np.nonzero(rows[:, 1])[0][0])
    rows[first, 1] = img.size - 3  # record runs past the end
    size = img.size
    src = torch.zeros(4 * size, dtype=torch.uint8, device=dev)
    src[:size] = torch.from_numpy(img).to(dev)
    src[size:2 * size] = torch.from_numpy(corrupt).to(dev)
    dst = torch.zeros(8 * size, dtype=torch.uint8, device=dev)
    m = hb.tab_part_redirect(cap["map_before"], cap["tab_old"], cap["tab_new"])
    d_maps = torch.from_numpy(m.view(np.int16)).to(dev)
    jobs = (hb.TabJob * 6)()
    spec = [  # src, src_len, keep, move, cap
        (0, size, 0, size, size),                      # good
        (size, size, 2 * size, 3 * size, size),        # corrupt record
        (3 * size + 8, size, 4 * size, 5 * size, size),  # source past the buffer
        (0, size, 6 * size, 7 * size, 70000),          # outputs too small for the data
        (4, size, 0, size, size),                      # misaligned source
        (0, size, 7 * size + 16, 0, size),             # keep past the buffer
    ]
    for j, (s, sl, k, mv, c) in zip(jobs, spec):
        j.src, j.src_len, j.keep, j.move, j.cap, j.map, j.tab_new = s, sl, k, mv, c, 0, cap["tab_new"]
        j.keep_type, j.move_type, j.status = 0x3E, 0xBE, 99
    d_jobs = torch.from_numpy(np.frombuffer(bytes(jobs), dtype=np.uint8).copy()).to(dev)
    prm = hb.TabParams(0, 0, 0, 1)
    rc = lib.shf_tab_copy_batch(src.data_ptr(), src.numel(), dst.data_ptr(), dst.numel(), d_jobs.data_ptr(), 6,
                                d_maps.data_ptr(), 1, ctypes.byref(prm), hb.MEM_DEVICE)
    assert rc == hb.ERR_ARG
    done = (hb.TabJob * 6).from_buffer_copy(d_jobs.cpu().numpy().tobytes())
    assert [done[i].status for i in range(6)] == [hb.OK] + [hb.ERR_ARG] * 5
    keep = dst[:size].cpu().numpy()
    kt, mt = tabcheck.observed_types(cap)
    want, _ = hb.tab_copy([img], [m], [cap["tab_new"]], keep_type=0x3E, move_type=0xBE)[0]
    assert np.array_equal(keep, want[:size])


def test_refs_repeating_one_large_record_fail(hb, dev):
    """A corrupt image whose 8192 refs all name one 2-MiB record: each ref is
    inside the image, their lengths sum to 16 GiB. The u32 size scans would
    wrap to exactly 0 per segment (2048 x 2 MiB = 2^32); the exact u64 total
    rejects the job -- status ERR_ARG, no fault, nothing past cap."""
    lib = hb.load()
    data_off = 24 + 512 * 16 * 8
    rec = 1 << 21  # SHF_DATA_TYPE + u32 key length + key + u32 value length (0) = 2 MiB
    kl = rec - 9
    img = np.zeros(data_off + rec, dtype=np.uint8)
    img[data_off] = 0x3E
    img[data_off + 1:data_off + 5] = np.frombuffer(np.uint32(kl).tobytes(), np.uint8)
    hdr = img[:24].view(np.uint32)
    hdr[:] = [img.size, img.size, 2 * 8192, 0, 1, rec]  # tab_data_free != 0: the length-word path
    rows = img[24:data_off].view(np.uint32).reshape(-1, 2)
    rows[:, 0] = 5 | (123 << 11)
    rows[:, 1] = data_off
    size = img.size
    src = torch.from_numpy(img).to(dev)
    dst = torch.zeros(size + 4096, dtype=torch.uint8, device=dev)
    jobs = (hb.TabJob * 1)()
    j = jobs[0]
    j.src, j.src_len, j.keep, j.move, j.cap, j.map, j.tab_new = 0, size, 0, 0, size, 0, 0xFFFF
    j.keep_type, j.move_type, j.status = 0x3E, 0x3E, 99
    d_jobs = torch.from_numpy(np.frombuffer(bytes(jobs), dtype=np.uint8).copy()).to(dev)
    prm = hb.TabParams(0, 0, 0, 1)
    rc = lib.shf_tab_copy_batch(src.data_ptr(), size, dst.data_ptr(), dst.numel(), d_jobs.data_ptr(), 1, None, 0,
                                ctypes.byref(prm), hb.MEM_DEVICE)
    assert rc == hb.ERR_ARG
    done = (hb.TabJob * 1).from_buffer_copy(d_jobs.cpu().numpy().tobytes())
    assert done[0].status == hb.ERR_ARG
    assert not dst[size:].any().item()  # nothing written past cap


def test_host_memory_entry_point(hb, dev):
    lib = hb.load()
    cap = fixture_caps()[1]
    img = np.array(cap["before"], dtype=np.uint8)
    m = hb.tab_part_redirect(cap["map_before"], cap["tab_old"], cap["tab_new"])
    size = img.size
    dst = np.zeros(2 * size, dtype=np.uint8)
    jobs = (hb.TabJob * 1)()
    j = jobs[0]
    j.src, j.src_len, j.keep, j.move, j.cap, j.map, j.tab_new = 0, size, 0, size, size, 0, cap["tab_new"]
    kt, mt = tabcheck.observed_types(cap)
    j.keep_type, j.move_type = kt, mt
    prm = hb.TabParams(1, cap["fixed_key_len"], cap["fixed_val_len"], cap["factor"])
    rc = lib.shf_tab_copy_batch(img.ctypes.data, size, dst.ctypes.data, dst.size, ctypes.addressof(jobs), 1,
                                m.ctypes.data, 1, ctypes.byref(prm), hb.MEM_HOST)
    assert rc == hb.OK and jobs[0].status == hb.OK
    tabcheck.check_capture(cap, dst[:size], dst[size:], 16)


@pytest.mark.parametrize("n_refs,kl,vl,seed", [
    (8192, (0, 0), (0, 0), 1),        # every ref used, minimal 9-B records (chunks straddle several)
    (300, (1000, 5000), (0, 3000), 2),  # few, large records (kilobytes: many chunks each)
    (4500, (16, 64), (8, 128), 3),      # the bench's shape
    (1, (5, 5), (5, 5), 4),             # a single record
    (0, (8, 8), (8, 8), 5),             # an empty tab
])
def test_synthetic_tabs_match_oracle(hb, dev, oracle, n_refs, kl, vl, seed):
    """Synthetic tabs (sharedhashfile_amd/tabgen.py) of very different shapes,
    parted and shrunk in one launch, against the CPU oracle: the kernel's
    segment boundaries, record lists and chunk gathers at their extremes."""
    from sharedhashfile_amd.tabgen import synth_tab

    img, m, old = synth_tab(seed, n_refs=n_refs, key_lo=kl[0], key_hi=kl[1], val_lo=vl[0], val_hi=vl[1])
    new = (old + 1000) % 2048
    m2 = hb.tab_part_redirect(m, old, new)
    got = hb.tab_copy([img, img], [m2, m2], [new, hb.TAB_NONE], keep_type=0x3E, move_type=0xBE)
    for (keep, move), tn in zip(got, [new, hb.TAB_NONE]):
        wk, wm = oracle.tab_split(img, m2, tn, cap=keep.size, keep_type=0x3E, move_type=0xBE)
        assert np.array_equal(keep, wk)
        if tn == hb.TAB_NONE:
            assert move is None
        else:
            assert np.array_equal(move, wm)


@pytest.mark.parametrize("factor", [1, 8, 20, 40])
def test_tab_size_growth_factor(hb, dev, oracle, factor):
    """The images' tab_size: closed form while every record times the growth
    factor fits a page (each SHF_TAB_APPEND growth is then one page), the
    growth replay otherwise (records of up to 201 B: factor 40 replays)."""
    from sharedhashfile_amd.tabgen import synth_tab

    img, m, old = synth_tab(7, n_refs=4500, key_lo=16, key_hi=64, val_lo=8, val_hi=128)
    new = (old + 77) % 2048
    m2 = hb.tab_part_redirect(m, old, new)
    got = hb.tab_copy([img, img], [m2, m2], [new, hb.TAB_NONE], factor=factor, keep_type=0x3E, move_type=0xBE)
    for (keep, move), tn in zip(got, [new, hb.TAB_NONE]):
        wk, wm = oracle.tab_split(img, m2, tn, False, 0, 0, factor, cap=keep.size, keep_type=0x3E, move_type=0xBE)
        assert np.array_equal(keep, wk)
        if tn != hb.TAB_NONE:
            assert np.array_equal(move, wm)


@pytest.mark.parametrize("case", ["packed", "deleted", "shared_pos", "first_gap"])
def test_lengths_from_positions_and_fallback(hb, dev, oracle, case):
    """Packed tabs (tab_data_free == 0) take each record's length from the
    next record's position; a deleted record (tab_data_free > 0), two refs
    sharing a position, or data not starting at the first record fall back to
    the length words. Every case against the oracle, which reads the words."""
    from sharedhashfile_amd.tabgen import TAB_DATA, TAB_HDR, synth_tab

    img, m, old = synth_tab(11, n_refs=3000, key_lo=8, key_hi=80, val_lo=0, val_hi=200)
    img = img.copy()
    rows = img[TAB_HDR:TAB_DATA].view(np.uint32).reshape(-1, 2)
    hdr = img[:TAB_HDR].view(np.uint32)
    used = np.nonzero(rows[:, 1])[0]
    if case == "deleted":  # the reference's delete: type byte, ref cleared, free bytes counted (shf.c:612-631)
        r = used[len(used) // 2]
        p = int(rows[r, 1])
        kl = int(img[p + 1:p + 5].view(np.uint32)[0])
        vl = int(img[p + 5 + kl:p + 9 + kl].view(np.uint32)[0])
        img[p] = 0x80
        rows[r, 1] = 0
        hdr[4] += 1 + 4 + kl + 4 + vl
        hdr[5] -= 1 + 4 + kl + 4 + vl
    elif case == "shared_pos":
        rows[used[7], 1] = rows[used[3], 1]
    elif case == "first_gap":  # the record at the start of the data is not referenced
        first = int(np.argmin(np.where(rows[:, 1] > 0, rows[:, 1], 0xffffffff)))
        rows[first, 1] = 0
    new = (old + 300) % 2048
    m2 = hb.tab_part_redirect(m, old, new)
    got = hb.tab_copy([img, img], [m2, m2], [new, hb.TAB_NONE], keep_type=0x3E, move_type=0xBE)
    for (keep, move), tn in zip(got, [new, hb.TAB_NONE]):
        wk, wm = oracle.tab_split(img, m2, tn, cap=keep.size, keep_type=0x3E, move_type=0xBE)
        assert np.array_equal(keep, wk), case
        if tn != hb.TAB_NONE:
            assert np.array_equal(move, wm), case
