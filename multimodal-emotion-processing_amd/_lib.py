"""ctypes binding of libmep_hip.so (include/mep.h).

The library is the product: there is no CPU or PyTorch fallback.  ``lib()`` raises if the
shared object is missing or cannot be loaded, and every launcher's return code is checked.
The ctypes structures below mirror include/mep.h field for field; tests/test_abi.py compiles a
C probe of the header with gcc and checks sizes and offsets against them.
"""
import ctypes
import os

import torch

PKG_DIR = os.path.dirname(os.path.abspath(__file__))

# Every MEP_* development switch the package reads, with the value in effect (bench.py prints it,
# so a stray variable on a box shows up in the line it changed).  Defaults are the product path.
SWITCHES = {}


def switch(name, default):
    """os.environ[name] or default, recorded in SWITCHES (with whether the environment set it)"""
    v = os.environ.get(name)
    SWITCHES[name] = {'value': default if v is None else v, 'from_env': v is not None}
    return default if v is None else v


def switches_from_env():
    """the MEP_* variables set in this process's environment (any, read or not)"""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith('MEP_')}


# MEP_LIB: development override (A/B experiments with variant builds); never set in normal use
LIB_PATH = switch('MEP_LIB', '') or os.path.join(PKG_DIR, 'libmep_hip.so')
# MEP_RFS: read by the library itself at each mep_rfw_epi_* call (csrc/rfw.hip rfs_on: 0 = the per-tile
# State_Transfer epilogues instead of the weight-stationary ones); recorded here for the bench line
switch('MEP_RFS', '1')

u64, i64, i32, f32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_float


class Rows(ctypes.Structure):
    _fields_ = [('ptr', u64), ('sB', i64), ('sT', i64), ('T', i32), ('_pad', i32)]


class GemmDesc(ctypes.Structure):
    _fields_ = [('x', Rows), ('y', Rows), ('w', u64), ('bias', u64), ('table', u64),
                ('ntok', i32), ('N', i32), ('K', i32), ('ldw', i32), ('w_nt', i32),
                ('accumulate', i32), ('relu', i32), ('alpha', f32), ('bf16', i32), ('ldt', i32)]


WGEMM_SUM_MAX = 4             # MEP_WGEMM_SUM_MAX


class GemmSumDesc(ctypes.Structure):
    _fields_ = [('src', GemmDesc * WGEMM_SUM_MAX), ('n_src', i32), ('_pad', i32), ('out', Rows)]


RF_FRONT_MAX_OUT = 12         # MEP_RF_FRONT_MAX_OUT
RF_FRONT_MAX_TILES = 96       # MEP_RF_FRONT_MAX_TILES


class RfFrontOut(ctypes.Structure):
    _fields_ = [('w', u64), ('y', Rows), ('N', i32), ('_pad', i32)]


class RfFrontDesc(ctypes.Structure):
    _fields_ = [('unify', GemmDesc), ('n_out', i32), ('n_tiles', i32), ('out', RfFrontOut * RF_FRONT_MAX_OUT),
                ('tile_map', ctypes.c_int16 * RF_FRONT_MAX_TILES)]


WG_MAX_B = 4


class WgradDesc(ctypes.Structure):
    _fields_ = [('a', Rows), ('b', Rows * WG_MAX_B), ('out', u64 * WG_MAX_B), ('kb', i32 * WG_MAX_B),
                ('ldo', i32 * WG_MAX_B), ('partial', u64), ('n_b', i32), ('ntok', i32), ('N', i32), ('Ktot', i32),
                ('tok_per_split', i32), ('n_split', i32), ('accumulate', i32), ('out_trans', i32),
                ('bf16', i32), ('_pad', i32)]


class AttnDesc(ctypes.Structure):
    _fields_ = [('q', Rows), ('k', Rows), ('v', Rows), ('x', Rows), ('mask', u64), ('mask_sB', i64),
                ('s_prev', u64), ('c', u64), ('s_out', u64), ('stats', u64),
                ('B', i32), ('H', i32), ('Tq', i32), ('Tk', i32)]


class AttnGenDesc(ctypes.Structure):
    _fields_ = [('f', AttnDesc), ('mask_sQ', i64), ('hd', i32), ('scale', ctypes.c_float)]


class AttnGenBwdDesc(ctypes.Structure):
    _fields_ = [('g', AttnGenDesc), ('dx', Rows), ('dq', Rows), ('dk', Rows), ('dv', Rows),
                ('ds_next', u64), ('ds_prev', u64), ('dc_partial', u64)]


class AttnBwdDesc(ctypes.Structure):
    _fields_ = [('f', AttnDesc), ('dx', Rows), ('dq', Rows), ('dk', Rows), ('dv', Rows),
                ('ds_next', u64), ('ds_prev', u64), ('dc_partial', u64)]


class EpiDesc(ctypes.Structure):
    _fields_ = [('q', Rows), ('x', Rows), ('xp', Rows), ('z', Rows), ('out', Rows),
                ('wp', u64), ('wm', u64), ('ln_w', u64), ('ln_b', u64), ('stats', u64), ('seed', u64),
                ('ntok', i32), ('D', i32), ('drop_p', f32), ('drop_stream', i32), ('out_h', Rows),
                ('drop_bits', u64)]


class EpiBwdDesc(ctypes.Structure):
    _fields_ = [('f', EpiDesc), ('dout', Rows), ('dout2', Rows), ('dz', Rows), ('dxp', Rows), ('dx', Rows),
                ('dq', Rows), ('ln_partial', u64), ('dq_accumulate', i32), ('pool_T', i32),
                ('pool_dpooled', u64), ('pool_argmax', u64), ('pool_C', i32), ('pool_Tq', i32),
                ('pool_t0', i32), ('pool_col', i32)]


class LnDesc(ctypes.Structure):
    _fields_ = [('x', Rows), ('y', Rows), ('dy', Rows), ('dx', Rows), ('w', u64), ('b', u64),
                ('stats', u64), ('partial', u64), ('ntok', i32), ('D', i32), ('dx_accumulate', i32),
                ('bf16', i32)]


class ColsumDesc(ctypes.Structure):
    _fields_ = [('partial', u64), ('out', u64), ('n_rows', i32), ('n_cols', i32), ('ld', i32),
                ('accumulate', i32)]


SUM_MAX_SRC = 16
SUM_BF16 = 2         # MEP_SUM_BF16: mep_sum_desc.accumulate bit, bf16 source / output rows


class SumDesc(ctypes.Structure):
    _fields_ = [('src', Rows * SUM_MAX_SRC), ('out', Rows), ('n_src', i32), ('ntok', i32), ('D', i32),
                ('accumulate', i32)]


class PoolDesc(ctypes.Structure):
    _fields_ = [('x', u64), ('dx', u64), ('pooled', u64), ('dpooled', u64), ('argmax', u64),
                ('B', i32), ('T', i32), ('C', i32), ('_pad', i32)]


class HeadDesc(ctypes.Structure):
    _fields_ = [('pooled0', u64), ('pooled1', u64), ('dpooled0', u64), ('dpooled1', u64), ('wc0', u64),
                ('wc1', u64), ('trans', u64), ('ln_w', u64), ('ln_b', u64), ('wo', u64), ('bo', u64),
                ('labels', u64), ('logits', u64), ('row_loss', u64), ('partial', u64),
                ('B', i32), ('F', i32), ('NC', i32), ('labels_are_float', i32), ('rdrop', i32),
                ('compute_grad', i32), ('loss_scale', f32), ('rdrop_pairs', i32), ('ext_dlogits', u64),
                ('mean_div', i32), ('_pad', i32), ('scale', u64)]


class RfEpiDesc(ctypes.Structure):
    _fields_ = [('q', Rows), ('x', Rows), ('xp', Rows), ('h', Rows), ('f1', Rows), ('f', Rows), ('out', Rows),
                ('wp', u64), ('w1', u64), ('b1', u64), ('w2', u64), ('b2', u64),
                ('ln1_w', u64), ('ln1_b', u64), ('ln2_w', u64), ('ln2_b', u64), ('a', u64), ('b', u64),
                ('stats', u64), ('ntok', i32), ('D', i32), ('FD', i32), ('_pad', i32), ('wparts', u64),
                ('wq_next', u64), ('qp_next', Rows), ('zero', Rows)]


class RfEpiBwdDesc(ctypes.Structure):
    _fields_ = [('f', RfEpiDesc), ('dout', Rows), ('dout2', Rows), ('df', Rows), ('df1', Rows), ('dxp', Rows),
                ('dx', Rows), ('dq', Rows), ('partial', u64), ('dq_accumulate', i32), ('_pad', i32),
                ('wq_in', u64), ('dqp_in', Rows)]


class WsplitDesc(ctypes.Structure):
    _fields_ = [('src', u64), ('dst', u64), ('R', i32), ('K', i32), ('ld', i32), ('trans', i32),
                ('nrows', i32), ('_pad', i32)]


def wsplit_bytes(R, K):
    """MEP_WSPLIT_BYTES: bytes of the three bf16 parts of an R x K weight (K padded to 32)"""
    return 3 * 2 * R * (-(-K // 32) * 32)


def rfw_part_offsets(D, FD):
    """MEP_RFW_PART_OFFSET: byte offsets of [Wp, W1, W2, Wp^T, W1^T, W2^T] parts and the total"""
    sizes = [wsplit_bytes(D, D), wsplit_bytes(FD, D), wsplit_bytes(D, FD), wsplit_bytes(D, D),
             wsplit_bytes(D, FD), wsplit_bytes(FD, D)]
    offs, o = [], 0
    for sz in sizes:
        offs.append(o)
        o += sz
    return offs, o


BF16_OPS, BF16_STORE = 1, 2   # MEP_BF16_OPS / MEP_BF16_STORE: the bf16 fields of the descriptors
COLSUM_NOT_GRAD = 2   # MEP_COLSUM_NOT_GRAD: a column sum that is not a gradient (left out of the folded norm)


def wsplit_desc(src, dst, N, K, ld, trans):
    """mep_wsplit descriptor of W' [N][K] (W'(n, k) = src[n * ld + k], or src[k * ld + n] when
    trans) with its rows padded to a multiple of 32 (the wave kernels' output-tile pairs)"""
    return WsplitDesc(src=src, dst=dst, R=-(-N // 32) * 32, K=K, ld=ld, trans=int(trans), nrows=N)


class PartsArena:
    """One device buffer holding the mep_wsplit parts of a plan's weights, and the mep_wsplit
    descriptors that refresh it (once per step, before the forward)."""

    def __init__(self):
        self.items, self.size = [], 0

    def _take(self, nbytes):
        off = self.size
        self.size += -(-nbytes // 256) * 256
        return off

    def add(self, src, N, K, ld, trans):
        """parts of W' [N][K]; returns the byte offset in the arena"""
        assert N > 0 and K > 0
        off = self._take(wsplit_bytes(-(-N // 32) * 32, K))
        self.items.append((off, src, N, K, ld, trans))
        return off

    def add_epi(self, D, FD, wp, w1, w2):
        """the six parts of a realformer epilogue (MEP_RFW_PART_OFFSET order, contiguous)"""
        offs, total = rfw_part_offsets(D, FD)
        base = self._take(total)
        for o, (src, N, K, ld, trans) in zip(offs, ((wp, D, D, D, 0), (w1, FD, D, D, 0), (w2, D, FD, FD, 0),
                                                    (wp, D, D, D, 1), (w1, D, FD, D, 1), (w2, FD, D, FD, 1))):
            self.items.append((base + o, src, N, K, ld, trans))
        return base

    def build(self, device):
        """allocate the arena; returns (buffer, DescArray of mep_wsplit descriptors, max units)"""
        buf = torch.zeros(max(self.size, 256), dtype=torch.uint8, device=device)
        base = buf.data_ptr()
        descs = [wsplit_desc(src, base + off, N, K, ld, trans) for (off, src, N, K, ld, trans) in self.items]
        units = max((d.R * (-(-d.K // 32)) * 4 for d in descs), default=0)
        return buf, DescArray(WsplitDesc, descs, device), units


def rf_partial_stride(D, FD):
    """MEP_RF_PARTIAL_STRIDE: floats per tile of mep_rf_epi_bwd's partial sums"""
    return 5 * D + FD + 2


class RfHeadDesc(ctypes.Structure):
    _fields_ = [('fc', u64), ('ln_w', u64), ('ln_b', u64), ('wc', u64), ('bc', u64), ('trans', u64),
                ('labels', u64), ('umask', u64), ('out', u64), ('h', u64), ('d12', u64), ('dfc', u64),
                ('row_loss', u64), ('partial', u64), ('ext_dout', u64),
                ('B', i32), ('P', i32), ('D', i32), ('compute_grad', i32), ('loss_scale', f32), ('_pad', i32),
                ('scale', u64)]


EVAL_MAX_MODELS, EVAL_MAX_CLASSES = 8, 16   # MEP_EVAL_MAX_* (include/mep.h)


class SweepDesc(ctypes.Structure):
    _fields_ = [('preds', u64 * EVAL_MAX_MODELS), ('weights', f32 * EVAL_MAX_MODELS), ('labels', u64),
                ('row_mask', u64), ('thresholds', u64), ('scores', u64), ('counts', u64),
                ('n_models', i32), ('N', i32), ('C', i32), ('n_thr', i32), ('P', i32), ('ld_pred', i32),
                ('ld_label', i32), ('post_div', f32), ('thr_per_class', i32), ('sorted', i32), ('hist', u64)]


WINDOW_MAX_DESC = 4   # MEP_WINDOW_MAX_DESC


class WindowDesc(ctypes.Structure):
    _fields_ = [('src', u64), ('segs', u64), ('sel', u64), ('start', u64), ('out', u64), ('mask', u64),
                ('n_out', i32), ('m_len', i32), ('d', i32), ('src_f64', i32), ('summary', i32), ('clean', i32),
                ('n_seq', i32), ('_pad', i32)]


class Seg(ctypes.Structure):
    _fields_ = [('offset', i64), ('length', i64)]


STRUCTS = {'mep_rows': Rows, 'mep_gemm_desc': GemmDesc, 'mep_gemm_sum_desc': GemmSumDesc, 'mep_wgrad_desc': WgradDesc,
           'mep_attn_desc': AttnDesc, 'mep_attn_bwd_desc': AttnBwdDesc, 'mep_attn_gen_desc': AttnGenDesc,
           'mep_attn_gen_bwd_desc': AttnGenBwdDesc, 'mep_epi_desc': EpiDesc,
           'mep_epi_bwd_desc': EpiBwdDesc, 'mep_ln_desc': LnDesc, 'mep_colsum_desc': ColsumDesc,
           'mep_sum_desc': SumDesc, 'mep_pool_desc': PoolDesc, 'mep_head_desc': HeadDesc, 'mep_seg': Seg,
           'mep_rf_epi_desc': RfEpiDesc, 'mep_rf_epi_bwd_desc': RfEpiBwdDesc, 'mep_rf_head_desc': RfHeadDesc,
           'mep_sweep_desc': SweepDesc, 'mep_window_desc': WindowDesc, 'mep_wsplit_desc': WsplitDesc}

P = ctypes.c_void_p
# name -> argtypes (all return int)
GROUPED = ['mep_gemm', 'mep_wsplit', 'mep_unify', 'mep_wgrad_reduce', 'mep_layernorm_fwd', 'mep_layernorm_bwd', 'mep_colsum', 'mep_sum_rows',
           'mep_pool_fwd', 'mep_pool_bwd']
GROUPED_T = ['mep_attn_fwd', 'mep_attn_bwd',      # + MEP_ATTN_* variant flags
             'mep_block_epi_fwd', 'mep_block_epi_bwd',  # + D (compiled variant)
             'mep_wgrad']                                # + MEP_PREC_BF16 (the bf16-path instance)
SIGNATURES = {name: [P, i32, i32, P] for name in GROUPED}
SIGNATURES.update({name: [P, i32, i32, i32, P] for name in GROUPED_T})
GROUPED_T2 = ['mep_rf_epi_fwd', 'mep_rf_epi_bwd', 'mep_rfw_epi_fwd', 'mep_rfw_epi_bwd']   # + D, FD (compiled variant)
SIGNATURES.update({name: [P, i32, i32, i32, i32, P] for name in GROUPED_T2})
HP = ctypes.POINTER(HeadDesc)
SIGNATURES.update({
    'mep_head_fwd_bwd': [HP, P],
    'mep_head_reduce': [HP, u64, u64, u64, u64, u64, u64, u64, u64, P],
    'mep_head_partial_stride': [i32],
    'mep_reduce_grads': [P, i32, i32, P, i32, i32, HP, u64, u64, u64, u64, u64, u64, u64, u64, P, P, P, P],
    'mep_reduce_grads_grid': [i32, i32, i32, i32, HP],
    'mep_reduce_grads_mapped': [P, P, HP, u64, u64, u64, u64, u64, u64, u64, u64, P, P, P, P, i32, P],
    'mep_wgrad_kt': [i32, i32],
    'mep_wgrad_occupancy': [i32],
    'mep_circle_loss_fwd': [P, P, i32, i32, i32, P, P, P],
    'mep_circle_loss_bwd': [P, P, i32, i32, P, P],
    'mep_clip_adam': [P, P, P, P, P, i32, i64, P, P, P, P, i32, P],
    'mep_clip_adam_ext': [P, P, P, P, P, i32, i64, P, P, P, P, i32, i32, P],
    'mep_seed_advance': [P, P],
    'mep_rf_head': [ctypes.POINTER(RfHeadDesc), P],
    'mep_threshold_sweep': [ctypes.POINTER(SweepDesc), P],
    'mep_assemble_windows': [ctypes.POINTER(WindowDesc), i32, P],
    'mep_tgemm': [P, i32, i32, i32, i32, P],
    'mep_wgemm': [P, i32, i32, i32, P],
    'mep_attn_general_fwd': [P, i32, i32, P],
    'mep_attn_general_bwd': [P, i32, i32, i32, P],
    'mep_wgemm_ws': [P, i32, i32, i32, i32, i32, P],
    'mep_wgemm_sum': [P, i32, i32, i32, P],
    'mep_rfw_front': [P, i32, i32, i32, P],
    'mep_abi_version': [],
    'mep_rf_rows': [i32, i32],
    'mep_last_error': [ctypes.c_char_p, ctypes.c_size_t],
    'mep_device_sync': [],
    'mep_hbm_probe': [P, P, i64, i32, i32, P],
    'mep_stamp': [P, i32, P],
    'mep_stamp_khz': [],
})

_LIB = None
ABI_VERSION = 7   # include/mep.h MEP_ABI_VERSION


def lib():
    """Load libmep_hip.so (raises OSError with a build hint if it is missing)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise OSError('libmep_hip.so not found at %s -- run __graft_entry__.build() '
                          '(make -C multimodal-emotion-processing_amd/csrc)' % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        if L.mep_abi_version() != ABI_VERSION:   # descriptor layouts would not match: fail loudly
            raise OSError('%s has ABI %d, this host expects %d: rebuild it' % (LIB_PATH, L.mep_abi_version(), ABI_VERSION))
        _LIB = L
    return _LIB


def last_error():
    buf = ctypes.create_string_buffer(512)
    lib().mep_last_error(buf, 512)
    return buf.value.decode(errors='replace')


def check(rc, what=''):
    if rc != 0:
        raise RuntimeError('libmep_hip %s failed (%d): %s' % (what, rc, last_error()))


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


# Optional per-launch hook (bench.py, scripts/bench_aux.py), None in normal operation: an object
# with begin(name, stream) / end(name, stream), called around every entry-point call (bench.py
# places its mep_stamp kernels there).
TIMER = None


def _run(name, run, stream):
    if TIMER is not None:
        TIMER.begin(name, stream)
    run()
    if TIMER is not None:
        TIMER.end(name, stream)


def call(name, *args, stream=None):
    fn = getattr(lib(), name)
    _run(name, lambda: check(fn(*args, stream_ptr(stream)), name), stream)


class DescArray:
    """A device-resident array of descriptors (kept alive by the plan that owns it)."""

    def __init__(self, struct, items, device, tail=None):
        """tail: int32 values stored right after the descriptors (the k_wgrad task map)."""
        self.n = len(items)
        self.struct = struct
        self.items = list(items)
        if self.n:
            arr = (struct * self.n)(*items)
            raw = bytes(arr) + (b'' if tail is None else bytes((ctypes.c_int32 * len(tail))(*tail)))
            host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
            self.dev = host.to(device)
        else:
            self.dev = None

    @property
    def ptr(self):
        return ctypes.c_void_p(self.dev.data_ptr() if self.dev is not None else 0)


def launch(name, descs, max_tiles, stream=None, threads=None, extra=()):
    """threads: the extra int argument of the GROUPED_T launchers (attention variant flags, or the
    epilogue width D); extra: the extra ints of the GROUPED_T2 launchers (D, FD)."""
    if descs.n == 0 or max_tiles <= 0:
        return
    fn = getattr(lib(), name)
    if threads is None and name == 'mep_wgrad':
        threads = getattr(descs, 'prec', 0)   # make_wgrad's precision
    ints = ([] if threads is None else [int(threads)]) + [int(x) for x in extra]
    ptr, n = descs.ptr, descs.n
    _run(name, lambda: check(fn(ptr, n, int(max_tiles), *ints, stream_ptr(stream)), name), stream)


ATTN_PREV, ATTN_SOUT, ATTN_SHORT, ATTN_LONG = 1, 2, 4, 8   # MEP_ATTN_* (include/mep.h)
PREC_BF16 = 0x10000   # MEP_PREC_BF16: bf16-operand products (attention flags, epilogue D argument)
ATTN_HD32 = 0x20000   # MEP_ATTN_HD32: head dim 32 attention forward (robot_demo)
ATTN_KV = 0x40000     # MEP_ATTN_KV: backward with k == v and dk == dv on every descriptor
ATTN_SPLITQ = 0x80000 # MEP_ATTN_SPLITQ: backward, Tk <= 64 descriptors on the workgroup-per-(b, h) kernel
ATTN_MAX_KCHUNKS = 8  # MEP_ATTN_MAX_KCHUNKS: the chunk-parallel backward (MEP_ATTN_KCHUNKS) up to 512 keys
ATTN_WIDE = switch('MEP_ATTN_WIDE', '1') != '0'   # 0: the key-chunk-serial kernel (A/B runs)


def attn_fwd_splitq(descs, min_units=1024):
    """(MEP_ATTN_SPLITQ, forward max_tiles with 16-query wave tasks) when the launch holds fewer
    (b, h) units than min_units, else (0, None)"""
    units = sum(d.B * d.H for d in descs)
    if not 0 < units < min_units:
        return 0, None
    return ATTN_SPLITQ, max(-(-(d.B * d.H * -(-d.Tq // 16)) // 4) for d in descs)


def attn_bwd_splitq(bdescs, min_units=1024):
    """MEP_ATTN_SPLITQ when the launch's Tk <= 64 descriptors hold fewer (b, h) units than
    min_units (one wave each on the short kernel would leave most of the 1024 SIMDs idle: cfg2's
    realformer layer has 64 x 6 = 384); 0 otherwise"""
    units = sum(b.f.B * b.f.H for b in bdescs if b.f.Tk <= 64)
    return ATTN_SPLITQ if 0 < units < min_units else 0


RFW = switch('MEP_RFW', '1') != '0'   # 0: the LDS-tiled f32-MFMA realformer kernels (A/B runs)
# realformer token GEMMs on the LDS-resident weight kernel (mep_wgemm_ws) from WGEMM_WS_MIN
# 16 x 32 output tiles per launch (State_Transfer, B x P x T tokens: 1133 -> 400 us per step),
# below it one wave per 16 tokens x 32 columns (mep_wgemm: cfg2's 3200-token launches, where the
# per-workgroup weight copy does not pay, 41.9 vs 42.6 us); MEP_WGEMM_WS=0: always mep_wgemm
WGEMM_WS = switch('MEP_WGEMM_WS', '1') != '0'
WGEMM_WS_MIN = 8192
WGEMM_WS_MAX_K = 320                               # mep_wgemm_ws: a column block's parts of every k pair in LDS
WGEMM_XVEC = 0x1                                   # MEP_WGEMM_XVEC


def wgemm_ws_fits(items):
    """mep_wgemm_ws takes the launch: enough tiles to pay for the per-workgroup weight copy, and
    every K within the LDS-resident column block (mep_wgemm has no K limit)"""
    return (WGEMM_WS and wgemm_tiles(items) >= WGEMM_WS_MIN and
            max(d.K for d in items) <= WGEMM_WS_MAX_K)


def wgemm_tiles(items):
    """16-token x 32-column output tiles of a token-GEMM launch (mep_wgemm's waves)"""
    return sum(-(-d.ntok // 16) * -(-d.N // 32) for d in items)


def wgemm_ws(descs, stream=None, x_padded=()):
    """mep_wgemm_ws over a DescArray of GemmDescs: MEP_WGEMM_XVEC when every X row view is
    16-byte aligned and K % 4 == 0 or the view's rows are padded (x_padded: x.ptr values whose
    buffers hold K rounded up to 4 readable floats per row)"""
    it = descs.items
    xvec = all(d.x.ptr % 16 == 0 and d.x.sB % 4 == 0 and d.x.sT % 4 == 0 and
               (d.K % 4 == 0 or d.x.ptr in x_padded) for d in it)
    call('mep_wgemm_ws', descs.ptr, descs.n, max(d.ntok for d in it), max(d.N for d in it), max(d.K for d in it),
         WGEMM_XVEC if xvec else 0, stream=stream)


def rf_bwd_rows(wave=None):
    """token rows per workgroup of the realformer epilogue backward, one row of its partial buffer
    each: mep_rfw_epi_bwd (wave-tiled, RFW) or mep_rf_epi_bwd -- the value the library was built
    with (mep_rf_rows), never a host constant"""
    return lib().mep_rf_rows(2 if (RFW if wave is None else wave) else 1, 0)


def rf_epi_rows(D, wave=False):
    """token rows per workgroup of mep_rf_epi_fwd (mep_rf_rows; 16 for mep_rfw_epi_fwd)"""
    return lib().mep_rf_rows(2 if wave else 0, D)
ATTN_MAX_DQ_TILES = (160 * 1024 // 4 - 2 * 4 * 64 * 16 - 4) // 256   # csrc/attn.hip backward LDS


def _uniform(flags, what):
    if any(flags) and not all(flags):
        raise ValueError('mep_attn: %s must be set for every descriptor of a launch or for none' % what)
    return bool(flags and flags[0])


def attn_geometry(descs):
    """AttnDesc list of one launch -> (fwd tiles, bwd tiles, fwd flags) following csrc/attn.hip:
    forward one wave per (b, h, 64-query chunk), 4 waves per workgroup; backward one workgroup per
    (b, h); flags = MEP_ATTN_* of the launch."""
    ft = bt = 0
    for d in descs:
        ft = max(ft, -(-(d.B * d.H * -(-d.Tq // 64)) // 4))
        bt = max(bt, d.B * d.H)
    # backward x extent a multiple of 32: the Tk > 64 kernels then put heads 4j .. 4j + 3 (or 2j,
    # 2j + 1) of a row on one XCD (csrc/attn.hip head_pair_order); the extra workgroups leave at once
    if any(d.Tk > 64 for d in descs):
        bt = -(-bt // 32) * 32          # a multiple of 32 for head quads (H % 4 == 0)
    flags = (ATTN_PREV if _uniform([d.s_prev != 0 for d in descs], 's_prev') else 0) | \
            (ATTN_SOUT if _uniform([d.s_out != 0 for d in descs], 's_out') else 0) | \
            (ATTN_SHORT if any(d.Tk <= 64 for d in descs) else 0) | (ATTN_LONG if any(d.Tk > 64 for d in descs) else 0)
    return ft, bt, flags


def attn_bwd_flags(bdescs):
    """AttnBwdDesc list of one launch -> MEP_ATTN_PREV | MEP_ATTN_SOUT (= ds_next present) |
    MEP_ATTN_DQ_TILES(largest ceil(Tq/16) among descriptors with Tk > 64: the query tiles whose dQ
    the backward carries across key chunks in LDS) | MEP_ATTN_KV when every descriptor has k == v
    and dk == dv (the same row view)"""
    same = lambda x, y: (x.ptr, x.sB, x.sT) == (y.ptr, y.sB, y.sT)  # noqa: E731
    kv = bool(bdescs) and all(same(b.f.k, b.f.v) and same(b.dk, b.dv) for b in bdescs)
    # Tk > 64: the chunk-parallel kernel (one wave per 64-key chunk, MEP_ATTN_KCHUNKS) up to
    # 64 * ATTN_MAX_KCHUNKS keys, else the key-chunk-serial kernel with the LDS-carried dQ
    kchunks = max([-(-b.f.Tk // 64) for b in bdescs if b.f.Tk > 64] or [0])
    wide = ATTN_WIDE and 2 <= kchunks <= ATTN_MAX_KCHUNKS
    dq_tiles = 0 if wide else max([-(-b.f.Tq // 16) for b in bdescs if b.f.Tk > 64] or [0])
    assert dq_tiles <= ATTN_MAX_DQ_TILES, 'mep_attn_bwd: Tq > %d with Tk > 64 exceeds the LDS' % (16 * ATTN_MAX_DQ_TILES)
    return (ATTN_PREV if _uniform([b.f.s_prev != 0 for b in bdescs], 's_prev') else 0) | \
           (ATTN_SOUT if _uniform([b.ds_next != 0 for b in bdescs], 'ds_next') else 0) | (dq_tiles << 8) | \
           ((kchunks << 20) if wide else 0) | \
           (ATTN_SHORT if any(b.f.Tk <= 64 for b in bdescs) else 0) | (ATTN_LONG if any(b.f.Tk > 64 for b in bdescs) else 0) | \
           (ATTN_KV if kv else 0)


N_CU = 256   # MI355X compute units


def epi_grid(ntok_max, n_desc):
    """Workgroups per descriptor of mep_block_epi_fwd / _bwd (csrc/block.hip): each workgroup
    owns a contiguous range of 16-token tiles of one block and stages that block's weights once,
    so the grid is sized to one workgroup per CU over all descriptors (never more workgroups than
    tiles)."""
    return max(1, min(-(-ntok_max // 16), N_CU // max(1, n_desc)))


def attn_dc_slots(B, H, Tk):
    """floats of the backward's dc_partial (one per (b, h, 64-key chunk))"""
    return B * H * -(-Tk // 64)


# ------------------------------------------------------------------ token GEMMs
TGEMM = switch('MEP_TGEMM', '1') != '0'   # 0: the mep_unify / mep_gemm kernels (A/B runs)
# mep_tgemm chunked (K in 32-wide LDS stages) wins where the weight is too large to keep resident
# (Ren-MME unify, K = 768 / 640: 153 -> 94 us at cfg5); at K <= 300 its per-chunk staging latency
# loses to the weight-stationary mep_unify / mep_gemm (cmu-mosei unify 22 vs 17 us; a
# resident-weight tgemm form measured 22.3 vs 17.4 us there, round 3, and was removed)
TGEMM_MIN_K = int(switch('MEP_TGEMM_MIN_K', '512'))
TGEMM_WT = 0x1                                     # MEP_TGEMM_WT: every descriptor has w_nt = 0
TGEMM_DMA = 0x4                                    # MEP_TGEMM_DMA (weight ring by LDS-DMA)
TGEMM_DMA_ON = switch('MEP_TGEMM_DMA', '1') != '0'


def tgemm_dma_ok(items):
    """MEP_TGEMM_DMA (include/mep.h) takes the chunked launches whose weights are stored [N][K]."""
    return all(d.w_nt for d in items)


def tgemm_mode(items):
    """Which mep_tgemm form can run these GemmDescs (include/mep.h): 'chunked' (some K >=
    TGEMM_MIN_K) or None (the mep_unify / mep_gemm kernels).  Needs N % 16 == 0
    with N in {32, 64, 96} or >= 128, one w_nt for the launch, 16-byte aligned y rows, bias and
    table rows."""
    if not TGEMM or not items or len({d.w_nt for d in items}) != 1:
        return None
    for d in items:
        if d.N % 16 or not (d.N in (32, 64, 96) or d.N >= 128):
            return None
        if d.y.ptr % 16 or d.y.sB % 4 or d.y.sT % 4 or d.bias % 16:
            return None
        if d.table and (d.table % 16 or (d.ldt or d.N) % 4):
            return None
        if d.ntok <= 0 or d.K <= 0:
            return None
    return 'chunked' if max(d.K for d in items) >= TGEMM_MIN_K else None


def tgemm_ok(items):
    return tgemm_mode(items) is not None


def gemm(name, descs, max_tiles, stream=None, prec=0, tgemm=True):
    """A token-GEMM launch (mep_gemm_desc array): the tiled split-bf16 kernel (mep_tgemm) when
    the descriptors allow it (and tgemm), else the named launcher (mep_unify / mep_gemm).  prec:
    MEP_PREC_BF16 for the bf16 path (mep_unify reads the per-descriptor bf16 field instead)."""
    if descs.n == 0:
        return
    mode = tgemm_mode(descs.items) if tgemm else None
    if mode is not None:
        flags = (prec & PREC_BF16) | (0 if descs.items[0].w_nt else TGEMM_WT)
        if any(d.bf16 for d in descs.items):
            flags |= PREC_BF16
        if TGEMM_DMA_ON and tgemm_dma_ok(descs.items):
            flags |= TGEMM_DMA
        call('mep_tgemm', descs.ptr, descs.n, max(d.ntok for d in descs.items), max(d.N for d in descs.items),
             flags, stream=stream)
        return
    launch(name, descs, max_tiles, stream)


def gemm_launcher(name, descs, tgemm=True):
    """Launch name a gemm() call is timed under (bench.py / roofline.py)."""
    return 'mep_tgemm' if tgemm and tgemm_ok(descs.items) else name
