"""Debug helper: LDS kernel at each DICE_LDS_G vs the oracle on the 600-template corpus; mismatch stats."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from licensee_amd._native import Scorer  # noqa: E402
from licensee_amd.corpus import TemplateCorpus  # noqa: E402
from licensee_amd.license import License  # noqa: E402
from licensee_amd.synth import SyntheticCorpus  # noqa: E402
from licensee_amd.synth_templates import synthetic_templates  # noqa: E402
from oracle.native import OracleScorer  # noqa: E402

tpl = synthetic_templates(License.all(hidden=True, pseudo=False), 600, seed=5)
corpus = TemplateCorpus(tpl)
fb = SyntheticCorpus(corpus).generate(0, 3000, seed=11, nthreads=8)
args = (corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length, corpus.is_cc,
        corpus.n_vocab)
orc = OracleScorer(*args)
eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=16)
for v in sys.argv[1:]:
    os.environ['DICE_LDS_G'] = v
    sc = Scorer(*args, device=0)
    best, ov, score = sc.match(fb, 98.0)
    bad = np.nonzero((best != eb) | (ov != eo) | (score != es))[0]
    print(f'G={v}: {len(bad)} mismatching files; first {bad[:10].tolist()}; '
          f'ov diff {(ov[bad].astype(np.int64) - eo[bad]).tolist()[:10]}; tiles {sorted(set((bad // 64).tolist()))[:20]}',
          flush=True)
    for _ in range(2):
        b2, o2, s2 = sc.match(fb, 98.0)
        print('  repeat identical:', np.array_equal(b2, best) and np.array_equal(o2, ov), flush=True)
