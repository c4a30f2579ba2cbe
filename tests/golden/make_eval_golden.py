"""Golden vectors for the evaluation loops, from the REFERENCE's own code.

The reference's ``test()`` functions (others/realformer.py:395-477, cmu-mosei/run.py:456-498)
are AST-extracted like the models (make_golden.py) and executed on the CPU over synthetic
precomputed model scores.  Three names in their namespace are supplied here, and only these:
  * ``data_loader`` yields the recorded synthetic batches in the reference's row format;
  * the models are callables returning the recorded scores of the batch (looked up by a marker
    stored in the first feature element);
  * ``torch.cuda.FloatTensor`` / ``LongTensor`` build CPU tensors, because this container has no
    GPU -- the loops' arithmetic is otherwise the reference's, on torch CPU;
  * ``tqdm`` is the identity.
Outputs: realformer's returned 18-tuple; cmu-mosei's printed accuracy / F1 lines (parsed).  The
inputs and outputs are written to tests/golden/eval_golden.npz (data only).

    python tests/golden/make_eval_golden.py
"""
import ast
import contextlib
import io
import os
import sys
import types

import numpy as np
import torch
from sklearn.metrics import accuracy_score, f1_score

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'


def reference_function(script, name, ns):
    path = os.path.join(REF, script)
    tree = ast.parse(open(path).read())
    node = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name][-1]
    exec(compile(ast.Module(body=[node], type_ignores=[]), path, 'exec'), ns)
    return ns[name]


def torch_on_cpu():
    """``torch`` with ``torch.cuda.FloatTensor`` / ``LongTensor`` producing CPU tensors."""
    mod = types.ModuleType('torch_cpu')
    mod.__dict__.update({k: getattr(torch, k) for k in dir(torch) if not k.startswith('__')})
    mod.cuda = types.SimpleNamespace(FloatTensor=torch.FloatTensor, LongTensor=torch.LongTensor)
    return mod


class ScoreModel:
    """Stands for a trained model: returns the recorded scores of the batch whose marker (first
    feature element) it is given."""

    def __init__(self, scores):
        self.scores = scores

    def eval(self):
        return self

    def __call__(self, linguistic, *rest):
        return torch.from_numpy(self.scores[int(linguistic.reshape(-1)[0])])


def realformer_case(rng, n_batches=3, B=4, P=6):
    batches, scores = [], [[], []]
    for k in range(n_batches):
        lens = rng.integers(1, P + 1, size=B)
        mask = (np.arange(P)[None, :] < lens[:, None]).astype(np.int64)
        mask[0, 2] = 0 if P > 3 else mask[0, 2]      # a hole: the reference's `break` skips the rest
        label = (rng.random((B, P, 6)) < 0.35).astype(np.int64)
        for m in range(2):
            scores[m].append(rng.normal(0.0, 0.8, (B, P, 6)).astype(np.float32))
        rows = []
        for i in range(B):
            l = np.zeros((P, 1, 1), np.float32)
            l[0, 0, 0] = k if i == 0 else 0.0
            rows.append((l, np.zeros((P, 1, 1), np.float32), np.zeros((P, 1, 1), np.float32), label[i],
                         np.ones((P, 1), np.float32), np.ones((P, 1), np.float32), np.ones((P, 1), np.float32),
                         mask[i]))
        batches.append(dict(rows=rows, label=label, mask=mask))
    ns = dict(torch=torch_on_cpu(), tqdm=lambda x: x, accuracy_score=accuracy_score, f1_score=f1_score,
              data_set=None, test_name_list=None, BATCH=B, P_LEN=P,
              data_loader=lambda data_set, names, batch_size: [b['rows'] for b in batches])
    test = reference_function('others/realformer.py', 'test', ns)
    best = test(ScoreModel(scores[0]), ScoreModel(scores[1]))
    return dict(rf_pred1=np.stack(scores[0]), rf_pred2=np.stack(scores[1]),
                rf_label=np.stack([b['label'] for b in batches]), rf_mask=np.stack([b['mask'] for b in batches]),
                rf_best=np.array(best, np.float64))


def cmu_case(rng, n_rows=40, n_models=4):
    scores = [[] for _ in range(n_models)]
    labels, batches = [], []
    for k in range(n_rows):
        label = (rng.random(7) < 0.4).astype(np.int64)
        labels.append(label)
        for m in range(n_models):
            scores[m].append(rng.normal(-0.2, 0.7, (1, 7)).astype(np.float32))
        l = np.zeros((2, 1, 1), np.float32)
        l[0, 0, 0] = k
        z = np.zeros((2, 1, 1), np.float32)
        batches.append([(l, z, z, np.ones(2, np.float32), np.ones(2, np.float32), np.ones(2, np.float32), label)])
    ns = dict(torch=torch_on_cpu(), tqdm=lambda x: x, accuracy_score=accuracy_score, f1_score=f1_score,
              test_name_list=None, label_dict=None, data_loader=lambda names, labels, batch_size: batches)
    test = reference_function('cmu-mosei/run.py', 'test', ns)
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        test(*[ScoreModel(s) for s in scores])
    printed = {}
    for line in out.getvalue().splitlines():
        key, val = line.split(':')
        printed[key.strip()] = float(val)
    order = ('happ', 'sadn', 'ange', 'fear', 'disg', 'surp')
    return dict(cmu_preds=np.stack([np.stack(s) for s in scores]), cmu_label=np.stack(labels),
                cmu_metrics=np.array([[printed[k + '_acc'], printed[k + '_f1']] for k in order], np.float64))


def main():
    rng = np.random.default_rng(2026)
    out = {}
    out.update(realformer_case(rng))
    out.update(cmu_case(rng))
    path = os.path.join(HERE, 'eval_golden.npz')
    np.savez_compressed(path, **out)
    print('wrote', path, os.path.getsize(path), 'bytes', out['rf_best'], out['cmu_metrics'].ravel())


if __name__ == '__main__':
    sys.exit(main())
