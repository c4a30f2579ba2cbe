"""Pin the CPU oracle against the golden vectors produced by the reference's own classes
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from tests import oracle_runner
from tests.golden import fixtures
from tests.gpu_util import check_grad_budget, close_or_spread, has_fp32_budget, post_budget_check

RTOL, ATOL = 2e-5, 2e-6


def close(a, b, rtol=RTOL, atol=ATOL):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), rtol=rtol, atol=atol)


@pytest.mark.parametrize('name', fixtures.names('model'))
def test_model_step(name):
    meta, gold = fixtures.load(name)
    out = oracle_runner.run_model_case(meta)
    close(out['logits'], gold['logits'])
    close(out['loss'], gold['loss'])
    close(out['gnorm'], gold['gnorm'], rtol=1e-5)
    budget = has_fp32_budget(gold)
    for k, g in out['grads'].items():
        if 'nograd/' + k in gold:
            assert g is None, k
            continue
        if budget:
            # rf_state_ref: the reference's own fp32 gradients scatter around the float64 values
            # (make_golden.py fp64_noise); the oracle is held to that budget against float64
            check_grad_budget(g, gold, k, meta['full'])
        elif meta['full']:
            close_or_spread(g, gold, 'grad/' + k, 1e-4, 1e-6)
        else:
            close(torch.linalg.vector_norm(g.double()), gold['gradnorm/' + k], rtol=1e-4, atol=1e-7)
            close(g.reshape(-1)[:256], gold['gradhead/' + k], rtol=1e-4, atol=1e-6)
    for k, p in out['post'].items():
        ref = gold['post/' + k] if meta['full'] else gold['posthead/' + k]
        got = p if meta["full"] else p.reshape(-1)[:256]
        if budget:
            # Adam's first step is ~lr * sign(g): entries whose gradient is within the fp32 noise
            # of zero may step the other way (gpu_util.post_budget_check)
            post_budget_check(got, gold, k, meta['full'])
        else:
            close(got, ref, rtol=1e-5, atol=2e-5)  # Adam: |update| <= lr; grads ~eps amplify rounding
    # (budget: the exempt entries' other step directions move logits2 by up to ~5e-5)
    close(out['logits2'], gold['logits2'], rtol=1e-3 if budget else 1e-4, atol=1e-4 if budget else 1e-5)


@pytest.mark.parametrize('name', fixtures.names('block'))
def test_block(name):
    meta, gold = fixtures.load(name)
    P, (qt, kvt, sp), y, s = oracle_runner.run_block_case(meta)
    close(y, gold['out'])
    close(s, gold['scores'], rtol=1e-6, atol=1e-4)
    _, _, _, _, g_out = fixtures.block_inputs(meta)
    obj = (y * torch.tensor(g_out)).sum()
    if meta['g_scores']:
        obj = obj + (s * torch.tensor(gold['g_scores'])).sum()
    obj.backward()
    close(qt.grad, gold['grad_q'], rtol=1e-4, atol=1e-5)
    close(kvt.grad, gold['grad_kv'], rtol=1e-4, atol=1e-5)
    if sp is not None:
        close(sp.grad, gold['grad_sprev'], rtol=1e-4, atol=1e-6)
    for k, p in P.items():
        if 'nograd/' + k in gold:
            assert p.grad is None
        else:
            close(p.grad, gold['grad/' + k], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize('name', fixtures.names('chain'))
def test_chain(name):
    meta, gold = fixtures.load(name)
    P, h, obj = oracle_runner.run_chain_case(meta)
    close(h, gold['out'])
    close(obj, gold['obj'], rtol=1e-5)
    for k, p in P.items():
        if 'grad/' + k in gold:
            close_or_spread(p.grad, gold, 'grad/' + k, 1e-4, 1e-6)


def test_robot_demo_inference():
    """oracle/robot_demo.py against the reference's robot_demo.py classes (4-model ensemble at its
    own configuration: D=192, 6 heads of 32, 2 layers, FFN 2, T = 25 / 100 / 100)."""
    from oracle import robot_demo as orb
    meta, gold = fixtures.load('robot_demo')
    inputs = fixtures.batch(meta)
    c = meta['ctor']
    preds = []
    for i, sd in enumerate(meta['seeds']):
        P = fixtures.params(dict(meta, seed=sd), requires_grad=False)
        with torch.no_grad():
            preds.append(orb.multi_class(P, *inputs, n_heads=c['n_heads'], n_layers=c['n_layers']))
        np.testing.assert_allclose(preds[-1].numpy(), gold['logits%d' % i], rtol=1e-4, atol=1e-5)
    ens = orb.ensemble(preds)
    np.testing.assert_allclose(ens.numpy(), gold['ensemble'], rtol=1e-4, atol=1e-5)
    probs = np.array([orb.probabilities(ens[r]) for r in range(ens.shape[0])])
    np.testing.assert_allclose(probs, gold['probs'], rtol=1e-5)
