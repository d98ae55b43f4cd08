"""Single-thread pure-Python restatement of the reference scoring (oracle/dice_oracle.py:
Ruby-Set-like Python sets, the same formula, sort and threshold) timed on a 10k-file subset of
the config-2 synthetic workload -- the interpreted-language reference point of BASELINE.md
("CPU baseline plan", item 3). Run in the build container only (not a GPU-box number):

    python tools/python_baseline.py [n_files]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from licensee_amd.corpus import TemplateCorpus  # noqa: E402
from licensee_amd.license import License  # noqa: E402
from licensee_amd.synth import SyntheticCorpus  # noqa: E402
from oracle import dice_oracle as O  # noqa: E402
from tests.helpers import oracle_templates  # noqa: E402


def main(n=10000):
    templates = License.all(hidden=True, pseudo=False)
    synth = SyntheticCorpus(TemplateCorpus(templates))
    otpl = oracle_templates(templates)
    files = []
    for i in range(n):
        text, cc, _ = synth.text(i)
        files.append((O.OracleFile(text), cc))    # wordset scan outside the timed loop
    t0 = time.perf_counter()
    matched = 0
    for f, cc in files:
        idx, _ = O.match(otpl, f, O.DEFAULT_THRESHOLD, cc_fp=cc)
        matched += idx >= 0
    dt = time.perf_counter() - t0
    print(f'{n} files x {len(otpl)} templates, 1 thread: {n / dt:.0f} files/s '
          f'({n * len(otpl) / dt:.3g} scores/s), {matched} matched')


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10000)
