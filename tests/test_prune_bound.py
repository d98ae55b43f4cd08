"""CPU check of the overlap bound the pruned match kernel uses (licensee_amd/csrc/dice_prune.hip).

ov_t = |Lf_t ∩ W_F| is bounded by m_t = sum over G word groups g of min(A_g, F_g), with word
group (p mod 64) / (64 / G) of u64 word p (the kernel uses G = 16; G = 32, measured as an A/B in
round 3, is checked too). The kernel evaluates it as
(sum_g A'_g + sum_g F_g - sum_g |A'_g - F_g|) / 2 over byte-clamped A'_g = min(A_g, 255), which
equals sum_g min(A_g, F_g) whenever every F_g <= 255 (else it uses m = |W_F ∩ V|). Checked here
in numpy against the C oracle's exact overlaps (oracle/dice_ref.c, content_helper.rb:128-133):
the identity, the bound, and that the bound's score is an upper bound of the exact score.
"""
import numpy as np


def _group_counts(bits, G=16):
    n, w64 = bits.shape
    per_word = np.unpackbits(bits.view(np.uint8), axis=1, bitorder='little').reshape(n, w64, 64).sum(2)
    grp = (np.arange(w64) % 64) // (64 // G)
    return np.stack([per_word[:, grp == g].sum(1) for g in range(G)], 1).astype(np.int64)


import pytest


@pytest.mark.parametrize('G', [16, 32])
def test_group_bound_identity_and_soundness(G):
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd.synth_templates import synthetic_templates
    from oracle.native import OracleScorer
    c = TemplateCorpus(synthetic_templates(License.all(hidden=True, pseudo=False), 130, seed=130))
    fb = SyntheticCorpus(c).generate(0, 2000, seed=131, nthreads=8)
    orc = OracleScorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab)
    mov, msc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, nthreads=8)
    A = _group_counts(c.lf_bits, G)               # [T, G]
    F = _group_counts(fb.bits, G)                 # [n, G]
    assert F.max() <= 255                         # synthetic license files stay on the byte path
    exact_min = np.minimum(A[None], F[:, None]).sum(2)
    A8 = np.minimum(A, 255)
    sad = np.abs(A8[None] - F[:, None]).sum(2)
    m = (A8.sum(1)[None] + F.sum(1)[:, None] - sad) // 2
    assert np.array_equal(m, exact_min)
    assert np.all(m >= mov)
    # the bound's score is an upper bound of the exact score (den > 0 here)
    d = np.abs(c.length[None].astype(np.int64) - fb.length[:, None])
    slack = c.length_slack[None].astype(np.int64)
    adj = np.where(slack < 0, d, np.maximum(d - slack, 0))
    den = (c.lf_size.astype(np.int64) - c.fields_set_size)[None] + fb.wordset_size[:, None] + adj // 4
    assert np.all(den > 0)
    assert np.all(m * 200.0 / den >= msc)
    # the kernel's den formula: max(|len - len_F| - max(slack, 0), 0) is the same adjusted delta
    assert np.array_equal(np.maximum(d - np.maximum(slack, 0), 0), adj)
