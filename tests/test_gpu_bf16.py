"""The bf16 path (include/mep.h MEP_PREC_BF16) against the fp32 reference golden vectors.

BASELINE cfg3 (cmu-mosei B=64 T=50) and cfg5 (Ren-MME T=300) are bf16 configurations.  On the bf16
path every matrix product of the encoders -- unify, attention scores / P.V / backward
contractions, block epilogue Linears, weight gradients -- takes plain bf16 operands (round to
nearest of the fp32 values, 2^-9 relative) with fp32 accumulation; storage, softmax, LayerNorm,
pool, head, loss and AdamW stay fp32.  It is selected the reference-side way, by running the
model under torch.autocast('cuda', dtype=torch.bfloat16), or by model.mep_precision = 'bf16'.

Reference and tolerance (bf16, separate from the fp32 path's 1e-4).  A bf16 execution picks other
max-pool argmaxes than the fp32 one wherever two time steps are within bf16 noise, and one flip
moves a block's whole gradient (heavy-tailed, different in every execution).  So the reference is
the pinned fp32 oracle run on the SAME routing: this path's own argmaxes (plan.argmax) replayed
through oracle/common.py POOL_ROUTE -- what is left is the bf16 arithmetic's continuous error.
The budget (tests/golden/bf16_budget.json, tests/golden/make_bf16_budget.py) is that error for
torch.autocast(bfloat16) of the same oracle against the fp32 oracle on autocast's routing, the
worst of 4 executions (the fixture and 3 with parameters scaled by 1 + 2^-18 N(0, 1)).  The HIP bf16
path must be about as accurate:
  logits max|d| / max|logit| and whole-gradient relative L2 error  <= 1.25 x budget
  loss relative error                                               <= 2 x budget + 1e-4
  EVERY gradient tensor's relative L2 error                         <= 1.5 x its budget
      (the scalar residual coefficients c: 4.3 x -- one ill-conditioned sum each; both factors
      are 2x the worst ratio measured on the five fixtures)
  post-AdamW parameters within lr/4 of the reference step           >= budget fraction - 0.01
and it must differ from the fp32 path (the bf16 kernels really ran).  The bf16 path stores its
activations as bf16 (include/mep.h MEP_PREC_BF16), as torch.autocast does between ops.
"""
import json
import os

import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import cmu_model, cuda_batch, ren_model

pytestmark = pytest.mark.gpu

CASES = ['cmu_small_l2', 'cmu_cfg3', 'ren_small', 'ren_ref', 'ren_cfg5']
# the replayed argmax of a column must lie within 2^-6 of the column's scale below its fp32 max
# (oracle/common.py POOL_ROUTE_RTOL): a bf16 near tie, not a wrong index
ROUTE_RTOL = 2.0 ** -6


def _budget(name):
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'bf16_budget.json')) as f:
        return json.load(f)[name]


def _model_and_batch(name, cuda):
    meta, gold = fixtures.load(name)
    if meta['family'] == 'cmu':
        model = cmu_model(meta, cuda)
        batch = cuda_batch(meta, cuda)
        return meta, gold, model, batch[:6], batch[6]
    model = ren_model(meta, cuda)
    inputs, labels = fixtures.batch(meta)
    return meta, gold, model, [t.to(cuda) for t in inputs], labels.to(cuda)


def _loss(meta, logits, labels):
    if meta['family'] == 'cmu':
        from mep_amd import cmu_mosei
        return cmu_mosei.multi_circle_loss(logits, labels).mean()
    from mep_amd import ren_mme
    return ren_mme.multi_loss(logits, labels) + ren_mme.rdrop_kl(logits)


def _routed_reference(meta, model, cuda):
    """the fp32 oracle's training step on this path's max-pool routing (the bf16 plan's argmax of
    the step just run, intensity then stimulation)"""
    from oracle import common as ocommon
    from tests import oracle_runner
    plans = list(model.mep_runner(cuda).plans.values())
    assert len(plans) == 1 and plans[0].bf16
    route = [a.long().cpu() for a in plans[0].argmax]
    ocommon.POOL_SEEN, ocommon.POOL_ROUTE, ocommon.POOL_ROUTE_RTOL = [], route, ROUTE_RTOL
    try:
        return oracle_runner.run_model_case(meta, steps=1)
    finally:
        ocommon.POOL_SEEN, ocommon.POOL_ROUTE, ocommon.POOL_ROUTE_RTOL = [], None, None


def _grad_errors(model, meta, gold, ref, budget):
    """(worst per-tensor error / its allowance, whole-gradient relative L2 error) against the
    routed reference's post-clip gradients (on the fixture's extent: whole tensors, or the first
    256 entries of the large fixtures); this path's gradients take the reference's clip factor."""
    coef = min(1.0 / (float(ref['gnorm']) + 1e-6), 1.0)
    pairs = []
    for k, p in model.named_parameters():
        if 'nograd/' + k in gold:
            assert p.grad is None, k
            continue
        n = gold[('grad/' if meta['full'] else 'gradhead/') + k].size
        g = (p.grad * coef).double().cpu().reshape(-1)[:n]
        r = ref['grads'][k].double().reshape(-1)[:n]
        pairs.append((k, g, r))

    def allow(k):
        # 1.5 x the tensor's budget: 2x the worst error / budget measured over every tensor of the
        # five fixtures (0.77, ren_small; round-5 session 14, RAWBUDGET lines), no absolute floor.
        # Named exemption: the residual coefficient c is ONE scalar whose gradient sums
        # B x H x Tq x Tk score terms dS * S_prev with heavy cancellation -- its relative error is
        # ill-conditioned (torch's own bf16 runs scatter it 3x between executions, bf16_budget
        # 'runs'); it gets 4.3 x its budget (2x the worst measured, 2.16 on cmu_small_l2)
        return (4.3 if k.endswith('.c') else 1.5) * budget['grads'][k]
    ratios = sorted(((float((g - r).norm() / r.norm()) / allow(k), k) for k, g, r in pairs), reverse=True)
    print('  worst tensors (error / allowance):', ', '.join('%s %.2f' % (k, e) for e, k in ratios[:3]))
    raw = sorted(((float((g - r).norm() / r.norm()) / budget['grads'][k], k) for k, g, r in pairs), reverse=True)
    print('  RAWBUDGET worst tensors (error / budget):', ', '.join('%s %.3f' % (k, e) for e, k in raw[:4]))
    assert ratios[0][0] <= 1.0, ratios[:5]          # every tensor (strict)
    gg = torch.cat([g for _, g, _ in pairs])
    rr = torch.cat([r for _, _, r in pairs])
    return ratios[0][0], float((gg - rr).norm() / rr.norm())


@pytest.mark.parametrize('name', CASES)
def test_bf16_autograd_vs_fp32_reference(name, cuda):
    meta, gold, model, args, labels = _model_and_batch(name, cuda)
    model.train()
    with torch.autocast('cuda', dtype=torch.bfloat16):
        logits = model(*args)
    runner = model.mep_runner(cuda)
    assert [k[-1] for k in runner.plans] == [True], 'autocast(bfloat16) did not select the bf16 plan'
    loss = _loss(meta, logits.float(), labels)
    loss.backward()
    ref = _routed_reference(meta, model, cuda)
    want = ref['logits'].double()
    e_logit = float((logits.detach().double().cpu() - want).abs().max() / want.abs().max())
    e_loss = abs(float(loss) - float(ref['loss'])) / abs(float(ref['loss']))
    bud = _budget(name)
    e_grad, e_all = _grad_errors(model, meta, gold, ref, bud)
    print('bf16 %s: logits %.2e (budget %.2e) loss %.2e (%.2e) grad all %.2e (%.2e)'
          % (name, e_logit, bud['logits'], e_loss, bud['loss'], e_all, bud['grad_all']))
    assert e_logit <= 1.25 * bud['logits'], (e_logit, bud['logits'])
    assert e_loss <= 2 * bud['loss'] + 1e-4, (e_loss, bud['loss'])
    assert e_all <= 1.25 * bud['grad_all'], (e_all, bud['grad_all'])
    assert e_grad <= 1.0, e_grad
    assert e_logit > 1e-6, 'bf16 logits equal the fp32 reference: the bf16 kernels did not run'


@pytest.mark.parametrize('name', ['cmu_cfg3', 'ren_ref'])
def test_bf16_engine_step(name, cuda):
    """One captured training step on the bf16 path (model.mep_precision): loss and post-AdamW
    parameters vs the fp32 reference step on the same routing."""
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    meta, gold, model, args, labels = _model_and_batch(name, cuda)
    model.mep_precision = 'bf16'
    model.train()
    lr = 1e-3
    opt = FusedAdamW(model, lr=lr)
    eng = TrainEngine(model, opt, clip=1.0, rdrop=meta['family'] == 'ren', graph=True)
    if meta['family'] == 'ren':
        from mep_amd import ren_mme
        args = ren_mme._pack(args)
    loss = float(eng.step(*args, labels).item())
    ref = _routed_reference(meta, model, cuda)
    bud = _budget(name)
    e_loss = abs(loss - float(ref['loss'])) / abs(float(ref['loss']))
    assert e_loss <= 2 * bud['loss'] + 1e-4, (e_loss, bud['loss'])
    n_ok = n_all = 0
    for k, p in model.named_parameters():
        n = gold[('post/' if meta['full'] else 'posthead/') + k].size
        got = p.detach().double().cpu().reshape(-1)[:n]
        r = ref['post'][k].double().reshape(-1)[:n]
        err = (got - r).abs()
        n_ok += int((err <= 0.25 * lr).sum())
        n_all += err.numel()
    frac = n_ok / n_all
    print('bf16 step %s: loss %.2e, params within lr/4: %.4f (budget %.4f)' % (name, e_loss, frac, bud['post_frac']))
    assert frac >= bud['post_frac'] - 0.01, (frac, bud['post_frac'])
    assert all(k[-1] for k in model.mep_runner(cuda).plans)
