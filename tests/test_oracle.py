"""Pin the CPU oracle (oracle/murmur3_oracle.c) to the reference's golden vectors.

The goldens were produced by the reference's own murmurhash3.c + shf.c
(tests/golden/make_golden.py); SMHasher's verification value is the external
known-answer test for MurmurHash3_x64_128.
"""
import hashlib

import numpy as np
import pytest

from sharedhashfile_amd.keygen import counter_keys, splitmix_bytes


def test_smhasher_verification(oracle, golden):
    assert oracle.smhasher() == int(golden["smhasher_verification"], 16) == 0x6384BA69


def test_golden_cases(oracle, golden):
    assert len(golden["cases"]) > 100
    for c in golden["cases"]:
        key = bytes.fromhex(c["key_hex"])
        h1, h2 = oracle.hash(key, c["seed"])
        assert (h1, h2) == (int(c["h1"], 16), int(c["h2"], 16)), c["name"]


def test_survey_golden_sample(oracle):
    # key bytes 0,1,... seed 12345.
    table = {0: ("230e8369e0320eaf", "51a8f4dd45f232be"), 1: ("92adc75db911d3be", "c67af23b1349fbab"),
             15: ("6bf888c77fd36eb1", "18c21109e3be9b28"), 16: ("75f6084eb51bf230", "7557dbd78cafc6ba"),
             17: ("94e3e4bb463b77a6", "030b337fc8025248"), 256: ("8acd2d7ac9a62791", "37b284f6726b7cd0"),
             512: ("1ca1ae7c9794934c", "e3adb19f091da7bf")}
    for n, (h1, h2) in table.items():
        assert oracle.hash(bytes(i & 0xFF for i in range(n))) == (int(h1, 16), int(h2, 16))


def test_readme_key_uid_parts(oracle, golden):
    c = next(c for c in golden["cases"] if c["name"] == "str_key")
    h = np.array([[int(c["h1"], 16), int(c["h2"], 16)]], dtype=np.uint64)
    p = int(oracle.uid_parts(h)[0])
    assert p == int(c["uid_parts"], 16)
    # "key" -> win=105, tab2=1848, row=222, rnd=1727318
    assert (p & 0xFF, (p >> 8) & 0x7FF, (p >> 19) & 0x1FF, (p >> 32) & 0x1FFFFF) == (105, 1848, 222, 1727318)


@pytest.mark.parametrize("width", [4, 16])
def test_counter_keys_test9_shape(oracle, golden, width):
    g = golden["counters"]["counter_w%d" % width]
    keys = counter_keys(g["count"], width)
    out = oracle.hash_fixed(keys)
    assert [("%016x" % v) for v in out[:64, 0]] == g["first_h1"]
    assert [("%016x" % v) for v in out[:64, 1]] == g["first_h2"]
    assert hashlib.sha256(out.astype("<u8").tobytes()).hexdigest() == g["sha256_of_hashes"]


@pytest.mark.parametrize("name", ["fixed_w16", "fixed_w256"])
def test_fixed_random(oracle, golden, name):
    g = golden["fixed"][name]
    flat = np.frombuffer(splitmix_bytes(g["key_len"] * g["count"], int(g["splitmix_stream"], 16)), dtype=np.uint8)
    assert hashlib.sha256(flat.tobytes()).hexdigest() == g["sha256_of_keys"]
    out = oracle.hash_fixed(flat, g["key_len"])
    assert hashlib.sha256(out.astype("<u8").tobytes()).hexdigest() == g["sha256_of_hashes"]
    out_mt = oracle.hash_fixed(flat, g["key_len"], threads=3)
    assert np.array_equal(out, out_mt)


def test_var_golden(oracle, golden_var):
    out = oracle.hash_var(golden_var["bytes"], golden_var["offsets"])
    assert np.array_equal(out, golden_var["hashes"])
    lens = np.diff(golden_var["offsets"].astype(np.int64))
    assert set((lens & 15).tolist()) == set(range(16))


def test_var_equals_fixed(oracle):
    keys = np.frombuffer(splitmix_bytes(48 * 100, 7), dtype=np.uint8)
    off = np.arange(101, dtype=np.uint64) * 48
    assert np.array_equal(oracle.hash_var(keys, off), oracle.hash_fixed(keys, 48))


def test_oracle_vs_compiled_reference_random():
    """Cross-check against oracle/_ref (the reference's code) where it was built."""
    from oracle.oracle_py import Oracle, reference_lib

    ref = reference_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    o = Oracle()
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 700, size=3000)
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    want = np.empty((lens.size, 2), dtype=np.uint64)
    ref.ref_hash_var(data.ctypes.data, off.ctypes.data, lens.size, want.ctypes.data)
    assert np.array_equal(o.hash_var(data, off), want)
