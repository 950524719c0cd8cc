"""LDS bank model check of the kernels' XOR/permutation swizzles (CPU only).

MI355X_MICROARCH.md §LDS: ds_read_b128 serves a wave in four 16-lane groups
{0-3,12-15,20-27}, {4-11,16-19,28-31} (+32 for the upper half), one LDS cycle per group when
the 16 lanes hit 16 distinct 16-B slots of the 256-B bank line. The formulas below mirror the
address math of csrc/kernels/gemm.hip (big_frag / lds_frag) and attention.hip (pf_off); each
MFMA fragment read must be conflict-free (the pre-fix 64-B-row XOR of the big GEMM was 2-way).
"""
import pytest

_G = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
_GROUPS = _G + [[lane + 32 for lane in g] for g in _G]


def _extra_cycles(addr):
    extra = 0
    for g in _GROUPS:
        slots = {}
        for lane in g:
            slots.setdefault((addr[lane] // 16) % 16, set()).add(addr[lane])
        extra += max(len(v) for v in slots.values()) - 1
    return extra


def big_swz(row):
    return (0x78 >> (2 * ((row >> 2) & 3))) & 3


def big_frag(row, chunk):           # 64-B rows: 256x32 bf16 K-tile of the big GEMM
    return row * 64 + ((chunk ^ big_swz(row)) << 4)


def tile_frag(row, chunk):          # 128-B rows: 64-wide K-tiles of the tile / decode GEMMs
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4)


def pf_off(row, ch):                # 256-B rows: D=128 K image of the prefill attention
    return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)))


@pytest.mark.parametrize("base", [0, 16, 48, 112])
def test_big_gemm_fragment_reads_conflict_free(base):
    assert _extra_cycles([big_frag(base + (lane & 15), lane >> 4) for lane in range(64)]) == 0


def test_old_big_gemm_xor_was_two_way():
    old = [(base + (lane & 15)) * 64 + (((lane >> 4) ^ (((base + (lane & 15)) >> 2) & 3)) << 4)
           for base in [0] for lane in range(64)]
    assert _extra_cycles(old) == 4          # every group 2-way


def test_big_swizzle_is_a_permutation_per_row():
    for row in range(256):
        assert sorted(c ^ big_swz(row) for c in range(4)) == [0, 1, 2, 3]


@pytest.mark.parametrize("base", [0, 16, 80])
@pytest.mark.parametrize("ks", [0, 1])
def test_tile_gemm_fragment_reads_conflict_free(base, ks):
    assert _extra_cycles([tile_frag(base + (lane & 15), 4 * ks + (lane >> 4)) for lane in range(64)]) == 0


@pytest.mark.parametrize("kt", [0, 1])
@pytest.mark.parametrize("ks", range(8))
def test_prefill_attention_k_reads_conflict_free(kt, ks):
    # S^T = K Q^T on 32x32x16: lane reads K row 32kt + (lane & 31), chunk 2ks + (lane >> 5)
    assert _extra_cycles([pf_off(32 * kt + (lane & 31), 2 * ks + (lane >> 5)) for lane in range(64)]) == 0


# paged-prefix prefill attention, LDS-staged kernel (attention_paged.hip): K page image of
# 256-B (bf16) / 128-B (fp8) rows, V^T page image of 64-B / 32-B rows
def pg_swz_k(key, fp8):
    return (((key >> 1) & 1) | (((key >> 3) & 3) << 1)) if fp8 else ((key & 3) | (((key >> 3) & 3) << 2))


def pg_k(lane, kt, ds, fp8):
    g, r = lane >> 4, lane & 15
    key = 8 * (r >> 2) + 4 * kt + (r & 3)
    c = (4 * (ds >> 1) + g) if fp8 else (4 * ds + g)
    return key * (128 if fp8 else 256) + 16 * (c ^ pg_swz_k(key, fp8))


def pg_v(lane, dt):                 # bf16: 16 B per lane
    g, r = lane >> 4, lane & 15
    d = 16 * dt + r
    return d * 64 + 16 * (g ^ ((d >> 1) & 3))


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("kt", [0, 1])
@pytest.mark.parametrize("ds", [0, 1, 2, 3])
def test_paged_prefill_k_reads_conflict_free(fp8, kt, ds):
    if fp8 and ds & 1:
        pytest.skip("an FP8 lane reads sub-steps ds and ds + 1 in one 16-B load")
    assert _extra_cycles([pg_k(lane, kt, ds, fp8) for lane in range(64)]) == 0


@pytest.mark.parametrize("dt", range(8))
def test_paged_prefill_v_reads_conflict_free(dt):
    assert _extra_cycles([pg_v(lane, dt) for lane in range(64)]) == 0
    # the first choice, (d >> 2) & 3, was conflict-free for 16 consecutive lanes but 2-way
    # under the hardware's lane groups
    old = [(16 * dt + (lane & 15)) * 64 + 16 * ((lane >> 4) ^ (((16 * dt + (lane & 15)) >> 2) & 3)) for lane in range(64)]
    assert _extra_cycles(old) == 4


def test_paged_prefill_swizzles_are_permutations():
    for row in range(32):
        assert sorted(c ^ pg_swz_k(row, False) for c in range(16)) == list(range(16))
        assert sorted(c ^ pg_swz_k(row, True) for c in range(8)) == list(range(8))
    for d in range(128):
        assert sorted(g ^ ((d >> 1) & 3) for g in range(4)) == [0, 1, 2, 3]
