"""The matrix-core dense prefix (dice_post_dense_mfma, licensee_amd/csrc/dice_post.hip) widens
bits to int8 0/1 bytes with widen_half: fragment dword k of lane half h is
(v >> (4 h + k)) & 0x01010101 for the k-step's 32-bit half v of a prefix word. The MFMA then sums
A[i][e] * B[e][j] over the 32 fragment elements e = 16 h + 4 k + byte of the two lane halves.

The overlap is exact iff, for both operands, the elements of one k-step are a permutation of the
step's 32 bits (each bit lands in exactly one element, and A and B use the same permutation, so each
product pairs one bit of the file with the same bit of the template). Checked here on the host:
the mapping is a bijection, and a numpy restatement of the widened dot product equals popcount(a & b)
on random words."""
import numpy as np


def widen_half(v: np.ndarray, h: int) -> np.ndarray:
    """Bytes (16 per value) of the fragment of lane half h, in element order (dword k, byte b)."""
    x = (v >> np.uint32(4 * h)).astype(np.uint32)
    dwords = [(x >> np.uint32(k)) & np.uint32(0x01010101) for k in range(4)]
    out = np.stack(dwords, axis=-1).view(np.uint8)          # little-endian: byte b of dword k
    return out.reshape(v.shape + (16,))


def test_bit_to_element_map_is_a_bijection():
    seen = {}
    for h in range(2):
        for k in range(4):
            for b in range(8 * 4 // 8):                     # 4 bytes per dword
                bit = 4 * h + k + 8 * b
                seen.setdefault(bit, []).append((h, k, b))
    assert sorted(seen) == list(range(32))
    assert all(len(v) == 1 for v in seen.values())


def test_widened_dot_product_is_popcount_of_and():
    rng = np.random.default_rng(7)
    a = rng.integers(0, 2**32, 4096, dtype=np.uint64).astype(np.uint32)
    b = rng.integers(0, 2**32, 4096, dtype=np.uint64).astype(np.uint32)
    # sparse words too (a template's word holds few bits)
    b[::3] &= rng.integers(0, 2**32, b[::3].size, dtype=np.uint64).astype(np.uint32)
    dot = np.zeros(a.size, np.int64)
    for h in range(2):
        dot += (widen_half(a, h).astype(np.int64) * widen_half(b, h).astype(np.int64)).sum(-1)
    pop = np.array([bin(int(x) & int(y)).count('1') for x, y in zip(a, b)])
    assert np.array_equal(dot, pop)
    # every byte is 0 or 1 (signed int8 operands of v_mfma_i32_32x32x32_i8)
    for h in range(2):
        assert set(np.unique(widen_half(a, h))) <= {0, 1}
