"""Run the CPU oracle on a golden fixture's recorded case (test infrastructure)."""
import torch

from oracle import cmu_mosei, common, realformer, ren_mme
from tests.golden import fixtures


def run_model_case(meta, steps=None):
    P = fixtures.params(meta)
    fam, ctor = meta['family'], meta['ctor']
    steps = meta['steps'] if steps is None else steps
    if fam == 'realformer':
        opt = common.AdamState(P.values(), lr=1e-3, weight_decay=0.0, decoupled=False)
    else:
        opt = common.AdamState(P.values(), lr=1e-3, weight_decay=0.01)
    out = {}
    b = fixtures.batch(meta)
    for step in range(steps):
        if fam == 'cmu':
            loss, logits, gn = cmu_mosei.train_step(P, opt, b, ctor['n_heads'], ctor['n_layers'])
        elif fam == 'ren':
            loss, logits, gn = ren_mme.train_step(P, opt, b[0], b[1], ctor['n_heads'], ctor['n_layers'])
        else:
            loss, logits, gn = realformer.train_step(P, opt, b, ctor['n_heads'], ctor['n_layers'])
        if step == 0:
            out.update(logits=logits, loss=loss, gnorm=gn,
                       grads={k: (None if p.grad is None else p.grad.clone()) for k, p in P.items()})
    with torch.no_grad():
        if fam == 'cmu':
            out['logits2'] = cmu_mosei.concat_trans(P, *b[:6], ctor['n_heads'], ctor['n_layers'])
        elif fam == 'ren':
            out['logits2'] = ren_mme.base_model(P, b[0], ctor['n_heads'], ctor['n_layers'])
        else:
            out['logits2'] = realformer.state_transfer(P, *b[:3], *b[4:7], ctor['n_heads'], ctor['n_layers'])
    out['post'] = {k: p.detach() for k, p in P.items()}
    return out


def block_dropout(meta, B, Tq, D):
    """A block fixture's dropout (meta['drop']): the counter-hash masks of seed advance(seed0),
    stream 0, site 0 then 1 -- what the standalone block draws in training mode"""
    d = meta.get('drop')
    if not d:
        return None
    from oracle import dropout as odrop
    seed, calls = odrop.seed_advance(d['seed0']), [0]

    def drop(t):
        site = calls[0] % 2
        calls[0] += 1
        return t * torch.from_numpy(odrop.block_mask(seed, 0, site, B, Tq, D, d['p']))
    return drop


def run_block_case(meta):
    P = fixtures.params(meta)
    q, kv, mask, s_prev, g_out = fixtures.block_inputs(meta)
    H = meta['ctor']['n_heads']
    qt = torch.tensor(q, requires_grad=True)
    kvt = torch.tensor(kv, requires_grad=True)
    sp = torch.tensor(s_prev, requires_grad=True) if s_prev is not None else None
    m = torch.tensor(mask) if mask is not None else None
    if meta['family'] == 'realformer':
        y, s = realformer.block(P, '', qt, kvt, m, H, s_prev=sp)
    else:
        norm = 'norm2' if meta['family'] == 'ren' else 'norm1'
        y, s = cmu_mosei.block(P, '', qt, kvt, m, H, s_prev=sp, norm=norm,
                               dropout=block_dropout(meta, q.shape[0], q.shape[1], q.shape[2]))
    return P, (qt, kvt, sp), y, s


def run_chain_case(meta):
    P = fixtures.params(meta)
    x, lm, G = fixtures.chain_inputs(meta)
    ctor = meta['ctor']
    w = P['unify_dimension.linguistic.weight'][:, :, 0]
    pos = P['linguistic_position.position_embeddings.weight']
    h0 = common.linear(torch.tensor(x), w) + pos[: meta['T']].unsqueeze(0)
    h, _ = realformer.encode_chain(P, '', h0, meta['n_layers'], ctor['n_heads'], torch.tensor(lm))
    obj = (h * torch.tensor(G)).mean()
    obj.backward()
    return P, h, obj
