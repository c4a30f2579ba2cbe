"""robot_demo.py inference on the GPU: the drop-in Multi_class at the
demo's own configuration (DIM 192, N_HEADS 6 -> head dim 32, N_LAYERS 2, FFN 2, T = 25 / 100 /
100), four models with the fixture's parameters, against the reference's logits, 4-model ensemble
and demo_output probabilities (tests/golden/robot_demo.npz, made by running robot_demo.py's own
classes).  Tolerances: logits / ensemble rtol 1e-4 (floor 1e-6 x max), probabilities 1e-5."""
import pytest
import torch

from tests.golden import fixtures, specs
from tests.gpu_util import OUT_ATOL_FRAC, assert_close

pytestmark = pytest.mark.gpu


def _models(meta, cuda):
    from mep_amd import robot_demo
    out = []
    for sd in meta['seeds']:
        m = robot_demo.Multi_class(**meta['ctor'])
        vals = specs.param_values(meta['shapes'], sd)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
        out.append(m.to(cuda).eval())
    return out


def test_robot_demo_ensemble(cuda):
    from mep_amd import robot_demo
    meta, gold = fixtures.load('robot_demo')
    models = _models(meta, cuda)
    inputs = [t.to(cuda) for t in fixtures.batch(meta)]
    with torch.no_grad():
        for i, m in enumerate(models):
            assert_close(m(*inputs), gold['logits%d' % i], 1e-4, OUT_ATOL_FRAC, 'model %d logits' % i)
    ens = robot_demo.ensemble_predict(models, *inputs)
    assert_close(ens, gold['ensemble'], 1e-4, OUT_ATOL_FRAC, 'ensemble')
    for r in range(ens.shape[0]):
        probs = robot_demo.demo_probabilities(ens[r].cpu())
        assert_close(list(probs.values()), gold['probs'][r], 1e-5, 0, 'probs row %d' % r)


def test_robot_demo_state_dict_and_guards(cuda):
    """Reference state_dict keys / shapes, and the loud failures outside the inference path."""
    from mep_amd import robot_demo
    meta, _ = fixtures.load('robot_demo')
    m = robot_demo.Multi_class(**meta['ctor'])
    assert {k: list(v.shape) for k, v in m.state_dict().items()} == meta['shapes']
    m = m.to(cuda)
    inputs = [t.to(cuda) for t in fixtures.batch(meta)]
    with pytest.raises(NotImplementedError):
        m.train()(*inputs)
    with pytest.raises(ValueError):
        m.eval()(inputs[0][:, :5], *inputs[1:])
