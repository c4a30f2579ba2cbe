"""Generate golden vectors from the REFERENCE implementation (run only in the build container).

The reference scripts cannot be imported (module top level imports mmsdk / tensorboard, reads
/home/... and starts training -- SURVEY.md F8), so this script parses each script with ``ast``
and executes only its class / function definitions and UPPERCASE constants, with ``device`` =
cpu and the constant overrides each case names.  It then runs the reference classes on seeded
inputs (tests/golden/specs.py) exactly as the reference ``train`` functions do -- forward, loss,
backward, ``clip_grad_norm_``, ``optim.AdamW`` / ``optim.Adam`` step -- and saves the outputs
(never the reference source) as ``tests/golden/<case>.npz``.

    python tests/golden/make_golden.py            # all cases
    python tests/golden/make_golden.py cmu_small  # one case

Fixture layout: ``meta`` (JSON: family, constants, ctor kwargs, batch spec, param shapes),
``logits``, ``loss``, ``gnorm`` (pre-clip global norm), ``grad/<key>`` (full grads, small cases)
or ``gradnorm/<key>`` + ``gradhead/<key>`` (first 256 entries, large cases), ``post/<key>`` /
``posthead/<key>`` (parameters after one optimizer step), ``logits2`` (forward after the step),
and block cases' ``out``, ``scores`` and input grads.
"""
import ast
import copy
import json
import math
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as optim

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import specs  # noqa: E402
from oracle import dropout as odrop  # noqa: E402

REF = '/root/reference'
SCRIPTS = {'cmu': 'cmu-mosei/run.py', 'realformer': 'others/realformer.py', 'ren': 'Ren-MME/run.py',
           'robot': 'robot_demo.py'}


def load_reference(family, overrides):
    path = os.path.join(REF, SCRIPTS[family])
    tree = ast.parse(open(path).read())
    ns = {'torch': torch, 'nn': nn, 'F': F, 'np': np, 'math': math, 'optim': optim,
          'device': torch.device('cpu')}
    consts = [n for n in tree.body if isinstance(n, ast.Assign)
              and all(isinstance(t, ast.Name) and t.id.isupper() for t in n.targets)]
    defs = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef))]
    exec(compile(ast.Module(body=consts, type_ignores=[]), path, 'exec'), ns)
    ns.update(overrides)
    exec(compile(ast.Module(body=defs, type_ignores=[]), path, 'exec'), ns)
    return ns


def set_params(model, seed, overrides=None):
    shapes = {k: list(v.shape) for k, v in model.state_dict().items()}
    vals = specs.param_values(shapes, seed, overrides)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return shapes


def leaf_overrides(model, leaf_values):
    """{state_dict key: value} for every key whose last component is in leaf_values (e.g. every
    residual coefficient ``c``)"""
    if not leaf_values:
        return None
    return {k: float(leaf_values[k.rsplit('.', 1)[-1]]) for k in model.state_dict()
            if k.rsplit('.', 1)[-1] in leaf_values}


def t(x):
    return torch.from_numpy(np.ascontiguousarray(x))


def dump_params(out, model, prefix, full):
    for k, p in model.named_parameters():
        v = p.detach().numpy().reshape(-1)
        if full:
            out[prefix + '/' + k] = p.detach().numpy().copy()
        else:
            out[prefix + 'head/' + k] = v[:256].copy()


def dump_grads(out, model, full):
    for k, p in model.named_parameters():
        if p.grad is None:
            out['nograd/' + k] = np.zeros(0, np.float32)
            continue
        g = p.grad.detach().numpy()
        if full:
            out['grad/' + k] = g.copy()
        else:
            out['gradnorm/' + k] = np.float64(np.linalg.norm(g.astype(np.float64)))
            out['gradhead/' + k] = g.reshape(-1)[:256].copy()


# ----------------------------------------------------------------------------------- cases

class MaskDrop(nn.Module):
    """Stand-in for one Attention_Block's nn.Dropout (Ren-MME/run.py:173): multiplies by the
    recorded keep-scale mask of the repo's counter hash (oracle/dropout.py) -- what nn.Dropout
    computes for that mask.  The block calls it twice per forward: site 0 on proj(x)
    (run.py:209), site 1 on norm2(minus(.)) (run.py:213)."""

    def __init__(self, block, seed, p):
        super().__init__()
        self.block, self.seed, self.p, self.calls = block, seed, p, 0

    def forward(self, x):
        if not self.training:
            return x
        site = self.calls % 2
        self.calls += 1
        B, T, D = x.shape
        return x * torch.from_numpy(odrop.block_mask(self.seed, self.block, site, B, T, D, self.p))


def case_model(name, family, consts, ctor, batch, full, seed, opt, steps=1, drop=None, noise64=False, leaf=None):
    """Whole-model train step(s) as the reference ``train`` performs them.  drop = (p, seed0):
    the blocks' dropout uses the masks of seed advance(seed0) (the engine advances the seed once
    before a training forward).  noise64: also run the reference's first step in float64 and store,
    per gradient, how far its own fp32 result lies from that (noise/<param>: max |g32 - g64| over
    the stored extent; noisenorm/<param>: the difference of the norms; noise/logits): the fp32
    rounding noise of the reference on this input, the floor of any fp32 parity check of it."""
    ns = load_reference(family, consts)
    torch.manual_seed(0)
    if family == 'cmu':
        model = ns['Concat_Trans'](**ctor)
    elif family == 'ren':
        model = ns['Base_model'](**ctor)
    else:
        model = ns['State_Transfer'](**ctor)
    overrides = leaf_overrides(model, leaf)
    shapes = set_params(model, seed, overrides)
    if drop is not None:
        p, seed0 = drop
        s1 = odrop.seed_advance(seed0)
        nl = ctor['n_layers']
        for e, enc in enumerate((model.intensity, model.stimulation)):
            for m, blk in enumerate(enc.multimodal_blocks):
                blk.drop = MaskDrop(e * 9 * nl + m, s1, p)
    model.train()
    model_for_noise = copy.deepcopy(model) if overrides else None
    if family == 'cmu':
        l, v, a, lm, vm, am, labels = specs.cmu_batch(**batch)
        args = [t(x) for x in (l, v, a, lm, vm, am)]
        labels = t(labels)
    elif family == 'ren':
        inputs, labels = specs.ren_batch(**batch)
        args = [t(x) for x in inputs]
        labels = t(labels)
    else:
        l, v, a, labels, lm, vm, am, um = specs.realformer_batch(**batch)
        args = [t(x) for x in (l, v, a, lm, vm, am)]
        labels, um = t(labels), t(um)
    if opt == 'adamw':
        optimizer = optim.AdamW(model.parameters(), lr=1e-3)
    else:
        optimizer = optim.Adam(model.parameters(), lr=1e-3)
    out = {}
    if noise64:
        out.update(fp64_noise(ns, family, model, args, labels, um if family == 'realformer' else None, full))
    for step in range(steps):
        optimizer.zero_grad()
        logits = model(*args)
        if family == 'cmu':
            loss = ns['multi_circle_loss'](logits, labels).mean()       # cmu-mosei/run.py:365-366
        elif family == 'ren':
            m_loss = ns['multi_loss'](logits, labels)                   # Ren-MME/run.py:331-334
            kl_0 = F.kl_div(F.logsigmoid(logits[::2]), torch.sigmoid(logits[1::2]), reduction='batchmean')
            kl_1 = F.kl_div(F.logsigmoid(logits[1::2]), torch.sigmoid(logits[::2]), reduction='batchmean')
            loss = m_loss + (kl_0 + kl_1) / 2
        else:
            loss = (ns['multi_circle_loss'](logits, labels) * um).mean()  # realformer.py:311-312
        loss.backward()
        gnorm = nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        if step == 0:
            out['logits'] = logits.detach().numpy()
            out['loss'] = np.float64(loss.item())
            out['gnorm'] = np.float64(gnorm.item())
            # grads are post-clip here; store the clip coefficient so tests can undo it
            out['clipcoef'] = np.float64(min(1.0, 1.0 / (gnorm.item() + 1e-6)))
            dump_grads(out, model, full)
        optimizer.step()
    if drop is not None:
        model.eval()                       # logits2: the no-dropout network after the step
    with torch.no_grad():
        out['logits2'] = model(*args).numpy()
    dump_params(out, model, 'post', full)
    meta = dict(kind='model', family=family, consts=consts, ctor=ctor, batch=batch, seed=seed,
                opt=opt, steps=steps, full=full, shapes=shapes)
    if overrides:
        meta['overrides'] = overrides
        out.update(f7_reference_noise(ns, family, model_for_noise, args, labels, full))

        def run(m):
            logits = m(*args)
            _loss_of(ns, family, logits, labels, None).backward()
            nn.utils.clip_grad_norm_(m.parameters(), 1.0)
            r = {'logits': logits.detach().numpy()}
            for k, p in m.named_parameters():
                if p.grad is not None:
                    g = p.grad.detach().numpy()
                    r[('grad/' if full else 'gradhead/') + k] = g if full else g.reshape(-1)[:256]
            return r
        out.update(perturbed_spread(model_for_noise, run, out, skip=overrides))
    if drop is not None:   # its own kind: the CPU oracle has no per-site masks
        meta.update(kind='model_drop', drop=dict(p=drop[0], seed0=drop[1], seed=odrop.seed_advance(drop[1])))
    return meta, out


def _loss_of(ns, family, logits, labels, um):
    if family == 'cmu':
        return ns['multi_circle_loss'](logits, labels).mean()
    if family == 'ren':
        kl_0 = F.kl_div(F.logsigmoid(logits[::2]), torch.sigmoid(logits[1::2]), reduction='batchmean')
        kl_1 = F.kl_div(F.logsigmoid(logits[1::2]), torch.sigmoid(logits[::2]), reduction='batchmean')
        return ns['multi_loss'](logits, labels) + (kl_0 + kl_1) / 2
    return (ns['multi_circle_loss'](logits, labels) * um).mean()


def fp64_noise(ns, family, model, args, labels, um, full, runs=6):
    """The fp32 rounding noise of this step's gradients on this input, as a budget for fp32 parity
    checks of it (realformer only).  On deep, gated inputs such as State_Transfer's (2-layer
    residual chains, ReLU FFNs, max-pools routing a column's gradient to one time step, a 6-step
    gate recurrence) single fp32 gradient entries land up to percent-level of a tensor's max away
    from the exact value, differently in every fp32 execution (a near tie resolved the other way).
    Stored:
      grad64/<param> (or grad64head/<param>): the reference's post-clip gradient in float64 from
        the fixture's parameters -- what fp32 executions are compared against;
      budget/<param>: the largest relative L2 error (over the stored extent) of a fp32 execution
        against its own float64 run, over `runs` executions of the reference and `runs` of the
        repo's CPU oracle (another fp32 summation order), each with the parameters scaled by
        1 + 2^-18 N(0, 1) except the first reference run.
    The caller's model is untouched."""
    import copy
    from oracle import realformer as orf
    assert family == 'realformer'
    gen = torch.Generator().manual_seed(20261018)

    def ref_grads(base, dt):
        m = copy.deepcopy(base).to(dt)
        a = [x.to(dt) if x.is_floating_point() else x for x in args]
        lab = labels.to(dt) if labels.is_floating_point() else labels
        _loss_of(ns, family, m(*a), lab, um.to(dt)).backward()
        nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        return {k: None if p.grad is None else p.grad.detach().double() for k, p in m.named_parameters()}

    def oracle_grads(base, dt):
        P = {k: v.detach().to(dt).clone().requires_grad_(True) for k, v in base.state_dict().items()}
        l, v, a, lm, vm, am = [x.to(dt) for x in args]
        out = orf.state_transfer(P, l, v, a, lm, vm, am, ctor_heads(base), ctor_layers(base))
        orf.loss_fn(out, labels.to(dt) if labels.is_floating_point() else labels, um.to(dt)).backward()
        torch.nn.utils.clip_grad_norm_([p for p in P.values() if p.grad is not None], 1.0)
        return {k: None if p.grad is None else p.grad.detach().double() for k, p in P.items()}

    def extent(g):
        return g if full else g.reshape(-1)[:256]

    out = {}
    for r in range(runs):
        base = copy.deepcopy(model)
        if r:
            with torch.no_grad():
                for p in base.parameters():
                    p.mul_(1 + 2.0 ** -18 * torch.randn(p.shape, generator=gen))
        g64 = ref_grads(base, torch.float64)
        if r == 0:
            for k, g in g64.items():
                if g is not None:
                    out[('grad64/' if full else 'grad64head/') + k] = extent(g).numpy()
        for g32 in (ref_grads(base, torch.float32), oracle_grads(base, torch.float32)):
            for k, g in g32.items():
                if g is None:
                    continue
                e = float((extent(g) - extent(g64[k])).norm() / max(float(extent(g64[k]).norm()), 1e-30))
                out['budget/' + k] = np.float64(max(e, float(out.get('budget/' + k, 0.0))))
    return out


def f7_reference_noise(ns, family, model, args, labels, full):
    """The reference's first step in float64 on the fixture's own parameters and inputs (F7
    fixtures, c <= -1): logits64 and grad64/<param> (post-clip, like grad/<param>).  Where the
    masked slots carry the row's maximum (c < -1) or lose their -1e8 (c = -1) the reference's fp32
    scores there are set by the fp32 rounding of ~1e8-sized terms, so its float64 run is a
    different function; the pair shows which entries depend on that rounding."""
    m = copy.deepcopy(model).double()
    a = [x.double() if x.is_floating_point() else x for x in args]
    lab = labels.double() if labels.is_floating_point() else labels
    logits = m(*a)
    _loss_of(ns, family, logits, lab, None).backward()
    nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    out = {'logits64': logits.detach().numpy()}
    for k, p in m.named_parameters():
        if p.grad is not None:
            g = p.grad.detach().numpy()
            out[('grad64/' if full else 'grad64head/') + k] = g if full else g.reshape(-1)[:256]
    return out


def ctor_heads(m):
    return m.feature.multimodal_blocks[0].n_heads


def ctor_layers(m):
    return len(m.feature.multimodal_blocks) // 9


def perturbed_spread(module, run, base, skip=(), runs=6, seed=20261019):
    """F7 fixtures: the reference's own fp32 sensitivity.  `run(copy)` evaluates the case on a copy
    of `module` and returns {name: array}; it is repeated on `runs` copies with every parameter
    scaled by 1 + 2^-18 N(0, 1) -- except the overridden ones in `skip` (c = -1 is a singular
    point: any other c leaves the masked slots ~1e8 * (1 + c) away from cancelling), and
    spread/<name> is the largest relative L2 distance of such a
    run from the unperturbed fp32 result `base` (spreadabs/<name>: the largest elementwise
    absolute distance).  Quantities that are sums of ~1e8-sized
    cancelling terms (the gradient of c through S_prev = -1e8 at masked keys) scatter by far more
    than fp32's epsilon between two such runs; a parity check of them can be no tighter."""
    gen = torch.Generator().manual_seed(seed)
    out = {}
    for _ in range(runs):
        m = copy.deepcopy(module)
        with torch.no_grad():
            for k, prm in m.named_parameters():
                noise = torch.randn(prm.shape, generator=gen)
                if k not in skip:
                    prm.mul_(1 + 2.0 ** -18 * noise)
        for k, v in run(m).items():
            b = np.asarray(base[k], np.float64)
            e = float(np.linalg.norm(np.asarray(v, np.float64) - b) / max(np.linalg.norm(b), 1e-30))
            out['spread/' + k] = np.float64(max(e, float(out.get('spread/' + k, 0.0))))
            a = float(np.abs(np.asarray(v, np.float64) - b).max()) if b.size else 0.0
            out['spreadabs/' + k] = np.float64(max(a, float(out.get('spreadabs/' + k, 0.0))))
    return out


def case_block(name, family, consts, ctor, B, Tq, Tk, seed, with_prev=True, g_scores=True, leaf=None,
               mask_kind='key', drop=None):
    """Standalone Attention_Block forward/backward with residual scores and an upstream
    gradient on both outputs (out, post-mask scores).  leaf: constant parameter overrides (the
    F7 fixtures' c <= -1); those also store the same computation in float64 (<key>64) and the
    reference's fp32 spread under parameter perturbation (perturbed_spread).  mask_kind: the mask
    form passed (specs.block_inputs).  drop = (p, seed0): the block in training mode with its
    nn.Dropout at p, on the masks of the repo's counter hash for seed advance(seed0), stream 0
    (MaskDrop: the standalone block advances its seed once per training forward)."""
    ns = load_reference(family, consts)
    blk = ns['Attention_Block'](**ctor)
    overrides = leaf_overrides(blk, leaf)
    shapes = set_params(blk, seed, overrides)
    if drop is not None:
        blk.drop = MaskDrop(0, odrop.seed_advance(drop[1]), drop[0])
        blk.train()
    D, H = ctor['dim'], ctor['n_heads']
    q, kv, mask, s_prev, g_out = specs.block_inputs(seed + 1, B, Tq, Tk, D, H, with_prev, mask_kind)
    rng = np.random.default_rng(seed + 2)
    g_s = (0.05 * rng.standard_normal((B, H, Tq, Tk))).astype(np.float32)

    def run(b, dt=torch.float32):
        qt, kvt = t(q).to(dt).requires_grad_(), t(kv).to(dt).requires_grad_()
        sp = t(s_prev).to(dt).requires_grad_() if with_prev else None
        y, s = b(qt, kvt, kvt, None if mask is None else t(mask).to(dt), sp)
        obj = (y * t(g_out).to(dt)).sum()
        if g_scores:
            obj = obj + (s * t(g_s).to(dt)).sum()
        obj.backward()
        r = {'out': y.detach().numpy(), 'scores': s.detach().numpy(), 'grad_q': qt.grad.numpy(),
             'grad_kv': kvt.grad.numpy()}
        if with_prev:
            r['grad_sprev'] = sp.grad.numpy()
        for k, p in b.named_parameters():
            if p.grad is not None:
                r['grad/' + k] = p.grad.numpy().copy()
        return r
    out = {'g_scores': g_s}
    base = run(blk)
    out.update({k: v for k, v in base.items() if not k.startswith('grad/')})
    dump_grads(out, blk, True)
    if overrides:
        fresh = copy.deepcopy(blk)
        fresh.zero_grad(set_to_none=True)
        for k, v in run(copy.deepcopy(fresh).double(), torch.float64).items():
            out[k.replace('grad/', 'grad64/') if k.startswith('grad/') else k + '64'] = v
        out.update(perturbed_spread(fresh, run, base, skip=overrides))
    meta = dict(kind='block', family=family, consts=consts, ctor=ctor, B=B, Tq=Tq, Tk=Tk,
                seed=seed, with_prev=with_prev, g_scores=g_scores, shapes=shapes, mask_kind=mask_kind)
    if overrides:
        meta['overrides'] = overrides
    if drop is not None:
        meta['drop'] = dict(p=drop[0], seed0=drop[1])
    return meta, out


def case_chain(name, consts, ctor, B, T, n_layers, seed, leaf=None):
    """realformer "text chain" (BASELINE cfg2): Conv1d unify of l + position embedding +
    ``n_layers`` residual blocks (multimodal_blocks[0..n_layers-1]); objective mean(out * G).
    leaf: constant parameter overrides (F7: c <= -1), stored with every layer's post-mask scores
    (scores<i>), the float64 twin (<key>64) and the reference's fp32 spread (perturbed_spread)."""
    ns = load_reference('realformer', consts)
    mc = ns['Multi_class'](**ctor)
    overrides = leaf_overrides(mc, leaf)
    shapes = set_params(mc, seed, overrides)
    rng = np.random.default_rng(seed + 1)
    lm = specs.masks_for(rng, (B,), T)
    x = specs.features(rng, (B, T, consts['L_DIM']), lm)
    G = rng.standard_normal((B, T, ctor['dim'])).astype(np.float32)

    def run(m, dt=torch.float32):
        xt = t(x).to(dt)
        lt = m.unify_dimension.linguistic(xt.transpose(1, 2)).transpose(1, 2)
        lt = lt + m.linguistic_position(lt)
        h, s = lt, None
        r = {}
        for i in range(n_layers):
            h, s = m.multimodal_blocks[i](h, lt, lt, t(lm).to(dt), s)
            if overrides:
                r['scores%d' % i] = s.detach().numpy()
        obj = (h * t(G).to(dt)).mean()
        obj.backward()
        r.update({'out': h.detach().numpy(), 'obj': np.float64(obj.item())})
        for k, p in m.named_parameters():
            if p.grad is not None:
                r['grad/' + k] = p.grad.numpy().copy()
        return r
    fresh = copy.deepcopy(mc)
    out = run(mc)
    if overrides:
        for k, v in run(copy.deepcopy(fresh).double(), torch.float64).items():
            out[k.replace('grad/', 'grad64/') if k.startswith('grad/') else k + '64'] = v
        out.update(perturbed_spread(fresh, run, {k: v for k, v in out.items() if '64' not in k}, skip=overrides))
    meta = dict(kind='chain', family='realformer', consts=consts, ctor=ctor, B=B, T=T,
                n_layers=n_layers, seed=seed, shapes=shapes)
    if overrides:
        meta['overrides'] = overrides
    return meta, out


def case_robot(name, ctor, batch, seeds):
    """robot_demo.py inference (robot_demo.py:597-622): four Multi_class models (parameters from
    ``seeds``) in eval mode under no_grad on one batch; each model's logits, their ensemble mean
    (pred_1 + pred_2 + pred_3 + pred_4) / 4 and demo_output's per-emotion probabilities
    sigmoids(pred[0][c], t_c) for every row."""
    ns = load_reference('robot', {})
    models, shapes = [], None
    for sd in seeds:
        m = ns['Multi_class'](**ctor)
        shapes = set_params(m, sd)
        models.append(m.eval())
    inputs = [t(x) for x in specs.robot_batch(**batch)]
    with torch.no_grad():
        preds = [m(*inputs) for m in models]
    pred = (preds[0] + preds[1] + preds[2] + preds[3]) / 4
    thr = (0.1, 0.1, -0.1, 0.0, 0.1, 0.0)     # happ sadn ange disg surp fear (robot_demo.py:609)
    probs = np.array([[ns['sigmoids'](pred[r][c], thr[c]) for c in range(6)] for r in range(pred.shape[0])])
    out = {'logits%d' % i: p.numpy() for i, p in enumerate(preds)}
    out.update(ensemble=pred.numpy(), probs=probs)
    meta = dict(kind='robot', family='robot', ctor=ctor, batch=batch, seeds=list(seeds), seed=seeds[0],
                shapes=shapes)
    return meta, out


CMU_C = dict(L_DIM=300, V_DIM=35, A_DIM=74, DROP=0.0)
REN_C = dict(L_DIM=768, V_DIM=640, A_DIM=205, DROP=0.0)


def rf_consts(T, ffn=2):
    return dict(L_DIM=300, V_DIM=35, A_DIM=74, DROP=0.0, FFN=ffn, L_LEN=T, V_LEN=T, A_LEN=T)


def cmu_ctor(dim, heads, layers, T=50):
    return dict(dim=dim, l_len=T, v_len=T, a_len=T, n_heads=heads, n_layers=layers, ffn=1)


CASES = {
    'cmu_small': lambda: case_model('cmu_small', 'cmu', CMU_C, cmu_ctor(32, 2, 1),
                                    dict(seed=11, B=5, T=[7, 9, 12]), True, 101, 'adamw', 2),
    'cmu_small_l2': lambda: case_model('cmu_small_l2', 'cmu', CMU_C, cmu_ctor(32, 2, 2),
                                       dict(seed=12, B=4, T=[6, 10, 8]), True, 102, 'adamw'),
    'cmu_cfg1': lambda: case_model('cmu_cfg1', 'cmu', CMU_C, cmu_ctor(96, 6, 1),
                                   dict(seed=13, B=8, T=50), False, 103, 'adamw'),
    'ren_small': lambda: case_model('ren_small', 'ren', REN_C, dict(dim=32, l_len=5, v_len=6, a_len=8,
                                    n_heads=2, n_layers=1, ffn=1),
                                    dict(seed=14, pairs=3, T=[5, 6, 8]), True, 104, 'adamw'),
    'ren_full': lambda: case_model('ren_full', 'ren', REN_C, dict(dim=128, l_len=40, v_len=76, a_len=96,
                                   n_heads=8, n_layers=1, ffn=1),
                                   dict(seed=15, pairs=2, T=[40, 76, 96]), False, 105, 'adamw'),
    # Ren-MME's DROP = 0.1 (Ren-MME/run.py:36) with the repo's counter-hash masks
    'ren_drop': lambda: case_model('ren_drop', 'ren', dict(REN_C, DROP=0.1), dict(dim=32, l_len=5, v_len=6, a_len=8,
                                   n_heads=2, n_layers=1, ffn=1),
                                   dict(seed=20, pairs=3, T=[5, 6, 8]), True, 115, 'adamw', drop=(0.1, 20261016)),
    # BASELINE cfg3 shape (B=64, T=50, D=96, H=6) with ragged masks and 'no_name' rows
    'cmu_cfg3': lambda: case_model('cmu_cfg3', 'cmu', CMU_C, cmu_ctor(96, 6, 1),
                                   dict(seed=17, B=64, T=50, no_name_rows=(0, 13, 40)), True, 112, 'adamw'),
    # the reference's own Ren-MME lengths (Ren-MME/run.py:28-30: L_LEN 40, V_LEN 76, A_LEN 275)
    'ren_ref': lambda: case_model('ren_ref', 'ren', REN_C, dict(dim=128, l_len=40, v_len=76, a_len=275,
                                  n_heads=8, n_layers=1, ffn=1),
                                  dict(seed=18, pairs=3, T=[40, 76, 275]), False, 113, 'adamw'),
    # BASELINE cfg5 shape: T=300 for every modality, d = (768, 640, 205)
    'ren_cfg5': lambda: case_model('ren_cfg5', 'ren', REN_C, dict(dim=128, l_len=300, v_len=300, a_len=300,
                                   n_heads=8, n_layers=1, ffn=1),
                                   dict(seed=19, pairs=2, T=[300, 300, 300]), True, 114, 'adamw'),
    # DROP = 0.1 at Ren-MME's width (D = 128, H = 8) with one modality past 64 steps: the long
    # (key-chunked) attention path between the dropout sites, every gradient in full
    'ren_drop_long': lambda: case_model('ren_drop_long', 'ren', dict(REN_C, DROP=0.1),
                                        dict(dim=128, l_len=8, v_len=12, a_len=80, n_heads=8, n_layers=1, ffn=1),
                                        dict(seed=22, pairs=2, T=[8, 12, 80]), True, 116, 'adamw',
                                        drop=(0.1, 20261017)),
    'rf_state_small': lambda: case_model('rf_state_small', 'realformer', rf_consts(6),
                                         dict(l_dim=300, v_dim=35, a_dim=74, dim=32, l_len=6, v_len=6,
                                              a_len=6, n_heads=2, n_layers=2, ffn=2),
                                         dict(seed=16, B=3, P=3, T=6), True, 106, 'adam'),
    # State_Transfer at the reference's own configuration (others/realformer.py:23-38: P_LEN 6
    # utterances, DIM 96, N_HEADS 6, N_LAYERS 2, FFN 2, L/V/A_LEN 50), gate recurrence :266-286
    'rf_state_ref': lambda: case_model('rf_state_ref', 'realformer', rf_consts(50),
                                       dict(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=50, v_len=50,
                                            a_len=50, n_heads=6, n_layers=2, ffn=2),
                                       dict(seed=23, B=8, P=6, T=50), False, 117, 'adam', noise64=True),
    'block_cmu': lambda: case_block('block_cmu', 'cmu', CMU_C, dict(dim=32, n_heads=2, ffn=1),
                                    3, 7, 11, 107),
    'block_cmu_noprev': lambda: case_block('block_cmu_noprev', 'cmu', CMU_C, dict(dim=32, n_heads=2, ffn=1),
                                           2, 9, 5, 108, with_prev=False, g_scores=False),
    'block_rf': lambda: case_block('block_rf', 'realformer', rf_consts(8), dict(dim=32, n_heads=2),
                                   3, 8, 10, 109),
    'rf_chain_small': lambda: case_chain('rf_chain_small', rf_consts(10),
                                         dict(l_dim=300, v_dim=35, a_dim=74, dim=32, l_len=10, v_len=10,
                                              a_len=10, n_heads=2, n_layers=2, ffn=2), 4, 10, 2, 110),
    # robot_demo.py's own configuration (DIM 192, N_HEADS 6 -> head dim 32, N_LAYERS 2, FFN 2,
    # L/V/A_LEN 25/100/100: robot_demo.py:35-43), 4-model ensemble
    'robot_demo': lambda: case_robot('robot_demo', dict(dim=192, l_len=25, v_len=100, a_len=100, n_heads=6,
                                                        n_layers=2, ffn=2),
                                     dict(seed=21, B=3, T=[25, 100, 100]), (121, 122, 123, 124)),
    'rf_chain_cfg2': lambda: case_chain('rf_chain_cfg2', rf_consts(50),
                                        dict(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=50, v_len=50,
                                             a_len=50, n_heads=6, n_layers=2, ffn=2), 8, 50, 2, 111),
    # the cfg2 bench shape itself (B = 64): the wave kernels' B = 64 launches parity-pinned
    'rf_chain_cfg2_b64': lambda: case_chain('rf_chain_cfg2_b64', rf_consts(50),
                                            dict(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=50, v_len=50,
                                                 a_len=50, n_heads=6, n_layers=2, ffn=2), 64, 50, 2, 112),
}

# F7: residual coefficients c <= -1.  The post-mask scores carry
# -1e8 at masked keys; c * S_prev flips them to about +1.5e8 (c = -1.5: after the mask term the
# masked slots hold ~+5e7, the row's maximum, and take the whole softmax) or cancels the mask
# term exactly (c = -1: masked slots score ~0 beside the kept keys): cmu-mosei/run.py:243-254,
# others/realformer.py:190-201.  Every c of the model is set (first-layer c take no gradient).
for _c, _tag in ((-1.5, 'm15'), (-1.0, 'm1')):
    CASES['cmu_f7_' + _tag] = (lambda c=_c, tag=_tag: case_model(
        'cmu_f7_' + tag, 'cmu', CMU_C, cmu_ctor(32, 2, 2), dict(seed=12, B=4, T=[6, 10, 8]), True, 102, 'adamw',
        leaf={'c': c}))
    CASES['rf_chain_f7_' + _tag] = (lambda c=_c, tag=_tag: case_chain(
        'rf_chain_f7_' + tag, rf_consts(10), dict(l_dim=300, v_dim=35, a_dim=74, dim=32, l_len=10, v_len=10,
                                               a_len=10, n_heads=2, n_layers=2, ffn=2), 4, 10, 2, 110,
        leaf={'c': c}))
    CASES['block_cmu_f7_' + _tag] = (lambda c=_c, tag=_tag: case_block(
        'block_cmu_f7_' + tag, 'cmu', CMU_C, dict(dim=32, n_heads=2, ffn=1), 3, 7, 11, 107, leaf={'c': c}))
    CASES['block_rf_f7_' + _tag] = (lambda c=_c, tag=_tag: case_block(
        'block_rf_f7_' + tag, 'realformer', rf_consts(8), dict(dim=32, n_heads=2), 3, 8, 10, 109, leaf={'c': c}))


# the standalone Attention_Block.forward surface beyond the models' [B, Tk] key masks
# (cmu-mosei/run.py:236-262, Ren-MME/run.py:171-214, others/realformer.py:182-209): mask=None,
# [B, Tq, Tk] masks, and Ren-MME's block in training mode with DROP = 0.1
CASES.update({
    'block_cmu_nomask': lambda: case_block('block_cmu_nomask', 'cmu', CMU_C, dict(dim=32, n_heads=2, ffn=1),
                                           3, 7, 11, 131, mask_kind='none'),
    'block_cmu_mask3': lambda: case_block('block_cmu_mask3', 'cmu', CMU_C, dict(dim=32, n_heads=2, ffn=1),
                                          3, 7, 11, 132, mask_kind='q3'),
    'block_cmu_mask3_long': lambda: case_block('block_cmu_mask3_long', 'cmu', CMU_C, dict(dim=64, n_heads=4, ffn=1),
                                               2, 9, 300, 133, mask_kind='q3'),
    'block_rf_nomask': lambda: case_block('block_rf_nomask', 'realformer', rf_consts(8), dict(dim=32, n_heads=2),
                                          3, 8, 10, 134, mask_kind='none'),
    'block_rf_mask3': lambda: case_block('block_rf_mask3', 'realformer', rf_consts(8), dict(dim=32, n_heads=2),
                                         3, 8, 10, 135, mask_kind='q3'),
    'block_ren_drop': lambda: case_block('block_ren_drop', 'ren', dict(REN_C, DROP=0.1),
                                         dict(dim=32, n_heads=2, ffn=1), 3, 7, 11, 136, drop=(0.1, 20261020)),
    'block_ren_drop_mask3': lambda: case_block('block_ren_drop_mask3', 'ren', dict(REN_C, DROP=0.1),
                                               dict(dim=128, n_heads=8, ffn=1), 2, 12, 40, 137, mask_kind='q3',
                                               drop=(0.1, 20261021)),
})


def main(names):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for name in names:
        meta, out = CASES[name]()
        out['meta'] = np.array(json.dumps(meta))
        path = os.path.join(HERE, name + '.npz')
        np.savez_compressed(path, **out)
        print('wrote', path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main(sys.argv[1:] or list(CASES))
