"""Inputs of tools/exp/wordset_bench.cpp: 2000 normalized config-2 synthetic texts (one per line,
native normalizer) and the vendored corpus vocabulary.
    python tools/exp/wordset_bench_inputs.py /tmp/wsb"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else '/tmp/wsb'
    os.makedirs(out, exist_ok=True)
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.native_host import HostPrep
    from licensee_amd.synth import SyntheticCorpus
    c = TemplateCorpus(License.all(hidden=True, pseudo=False))
    hp = HostPrep(c)
    sc = SyntheticCorpus(c)
    with open(os.path.join(out, 'texts.txt'), 'w', encoding='utf-8') as fh:
        for i in range(2000):
            t = hp.normalize(sc.text(i)[0], 'LICENSE')
            if t is not None:
                fh.write(t.replace('\n', ' ') + '\n')
    with open(os.path.join(out, 'vocab.txt'), 'w', encoding='utf-8') as fh:
        fh.write('\n'.join(c.vocab) + '\n')


if __name__ == '__main__':
    main()
