"""TEST INFRASTRUCTURE ONLY -- the repo's dropout masks restated on the host (numpy uint64).

The reference draws nn.Dropout masks from torch's CPU RNG (Ren-MME/run.py:173,209,213), which a
GPU kernel cannot reproduce.  The HIP path instead derives every keep/drop decision from a
counter hash of (seed, dropout site, element index) (csrc/common.h drop_scale, seed stepped by
csrc/optim.hip k_seed), so a mask is a pure function of the seed.  This module restates that
function; tests/golden/make_golden.py uses it to run the REFERENCE Base_model with its nn.Dropout
layers replaced by "multiply by this mask" -- exactly what nn.Dropout computes for a given mask
(input * bernoulli / (1 - p)) -- so the fixture pins where the masks apply, their 1/(1-p) scale
and the gradient routing through them, while the mask statistics are checked as properties
(keep rate, scale) in tests/test_gpu_ren.py (test_dropout_mask_statistics).

Site numbering (trimodal.py _epi_desc, drop_stream = block index): block j of encoder e (0 =
intensity, 1 = stimulation) with n_layers per chain has index (e * 9 + chain) * n_layers + layer =
e * 9 * n_layers + (module index in multimodal_blocks); its site 0 is drop(proj(x))
(Ren-MME/run.py:209), site 1 drop(norm2(minus(.))) (run.py:213); stream = 2 * block + site.
Element index = token * D + feature, token = (row0 + b) * Tq + t, where row0 is the global index
of a data-parallel share's first row (0 on one GPU): the ranks together draw the full batch's masks.
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _mix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over='ignore'):
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xBF58476D1CE4E5B9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x


def seed_advance(seed):
    """csrc/optim.hip k_seed: seed <- mix64(seed + golden)."""
    with np.errstate(over='ignore'):
        return int(_mix64(np.uint64(seed) + GOLDEN))


def _lowbias32(x):
    x = np.asarray(x, dtype=np.uint32)
    with np.errstate(over='ignore'):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7FEB352D)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846CA68B)
        x = x ^ (x >> np.uint32(16))
    return x


def keep_scale(seed, stream, idx, p):
    """float32 keep-scale (0 or 1/(1-p)) of elements ``idx`` (uint64 array) of dropout stream
    ``stream`` -- csrc/common.h drop_scale: the stream key is the low 32 bits of one 64-bit mix of
    (seed, stream); an element hashes its index halves with the 32-bit lowbias32 mix."""
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over='ignore'):
        key = np.uint32(int(_mix64(np.uint64(seed) ^ (GOLDEN * np.uint64(stream + 1)))) & 0xFFFFFFFF)
        lo = (idx & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (idx >> np.uint64(32)).astype(np.uint32)
        h = _lowbias32(lo ^ _lowbias32(hi ^ key))
    u = (h >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    p32 = np.float32(p)
    scale = np.float32(1.0) / (np.float32(1.0) - p32)
    return np.where(u >= p32, scale, np.float32(0.0)).astype(np.float32)


def block_mask(seed, block, site, B, Tq, D, p, row0=0):
    """[B, Tq, D] keep-scale mask of one dropout site of one block (rows row0 .. row0 + B - 1 of
    the global batch)."""
    idx = np.arange(row0 * Tq * D, (row0 + B) * Tq * D, dtype=np.uint64)
    return keep_scale(seed, 2 * block + site, idx, p).reshape(B, Tq, D)
