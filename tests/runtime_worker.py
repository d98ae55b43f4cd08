"""Child process for tests/test_runtime.py: liblicensee_dice.so loaded BEFORE torch.

    python tests/runtime_worker.py <mode>

mode 'shared' : the loader maps the HIP runtime torch uses first (licensee_amd._native default)
mode 'second' : LICENSEE_DICE_HIP_RUNTIME='' -- the library binds /opt/rocm's runtime, then torch
                maps its own copy; dice_create must refuse with a clear message.
mode 'stub'   : LICENSEE_DICE_HIP_RUNTIME (set by the test) names a runtime whose soname differs from
                the library's (a torch built for another ROCm major): the loader must skip it, so
                only the library's own runtime is mapped and dice_create works (no torch import).
Prints one JSON line: the distinct libamdhip64 files mapped, dice_create's outcome, and (on a GPU,
mode 'shared') the mismatches of a torch-stream batch match against the oracle."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mapped_runtimes():
    seen = {}
    with open('/proc/self/maps') as fh:
        for line in fh:
            parts = line.split()
            if len(parts) >= 6 and os.path.basename(parts[5]).startswith('libamdhip64.so'):
                st = os.stat(parts[5])
                seen[(st.st_dev, st.st_ino)] = parts[5]
    return sorted(seen.values())


def main():
    mode = sys.argv[1]
    if mode == 'second':
        os.environ['LICENSEE_DICE_HIP_RUNTIME'] = ''
    from licensee_amd import _native
    _native.load_library()                        # the library first, no torch yet
    if mode == 'stub':
        gpu = None
        out = {'mode': mode, 'runtimes': mapped_runtimes(), 'torch_gpu': gpu,
               'decision': _native.preload_decision()[1]}
    else:
        import torch                              # torch after it
        gpu = torch.cuda.is_available()
        out = {'mode': mode, 'runtimes': mapped_runtimes(), 'torch_gpu': gpu}
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    c = TemplateCorpus(License.all(hidden=True, pseudo=False))
    try:
        sc = _native.Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc,
                            c.n_vocab)
        out['create'] = 'ok'
    except _native.DiceError as e:
        out['create'] = str(e)
        print(json.dumps(out))
        return
    if gpu:
        import numpy as np

        from licensee_amd.synth import SyntheticCorpus
        from oracle.native import OracleScorer
        f = SyntheticCorpus(c).generate(0, 5000, seed=7)
        stream = torch.cuda.Stream()
        b = sc.batch(f.n)
        b.upload(f, stream.cuda_stream)
        b.match(98.0, stream.cuda_stream)
        best, ov, score = b.download_match(stream.cuda_stream)
        orc = OracleScorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab)
        eb, eo, es = orc.match(f.bits, f.wordset_size, f.length, f.cc_false_positive, 98.0, nthreads=4, mode=0)
        out['mismatches'] = int(np.sum(best != eb) + np.sum(ov != eo) + np.sum(score != es))
        # torch still sees and uses the device after the library's context exists
        out['torch_sum'] = float(torch.arange(10, device='cuda', dtype=torch.float32).sum())
        b.close()
    sc.close()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
