"""ctypes binding of libsamplernn_hip.so (the C ABI in include/samplernn_hip.h).

This is the ONLY compute path of the drop-in model.py / nn.py / utils.py / optim.py:
there is no PyTorch or CPU fallback for device tensors.  If the library is missing or
fails to load, `lib()` raises -- loudly -- and so does every op that needs it.
PyTorch is used for device memory, streams and autograd bookkeeping only.
"""
import ctypes
import sys
import time
import os
import weakref

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libsamplernn_hip.so')

F32, BF16 = 0, 1
MAX_TIERS, MAX_RNN = 6, 4

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float
_D = ctypes.c_double
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t

# name -> argument types (all return int status)
_SIGS = {
    'srnn_uquantize_f32': [_P, _P, _L, _I, _P],
    'srnn_uquantize_f64': [_P, _P, _L, _I, _P],
    'srnn_udequantize': [_P, _P, _L, _I, _F, _I, _P],
    'srnn_udequantize2d': [_P, _L, _P, _I, _I, _I, _F, _I, _P],
    'srnn_uquantize_f64_host': [_P, _P, _L, _I],
    'srnn_uquantize_f32_host': [_P, _P, _L, _I],
    'srnn_udequantize_host': [_P, _P, _L, _I],
    'srnn_gemm': [_I, _I, _I, _I, _I, _I, _I, _F, _P, _L, _L, _P, _L, _L, _F, _P, _L, _L, _P, _L,
                  _L, _P, _I, _I, _I, _I, _P, _L, _P],
    'srnn_gemm_bits': [_I, _I, _I, _I, _I, _I, _I, _F, _P, _L, _P, _L, _F, _P, _L, _P, _L, _P, _I,
                       _I, _I, _P, _L, _P, _L, _P],
    'srnn_relu_bits': [_I, _P, _L, _I, _I, _P, _L, _P],
    'srnn_mlp_l1_bits': [_P, _P, _L, _I, _I, _I, _P, _L, _P, _L, _I, _I, _I, _P, _L, _P],
    'srnn_gru_cell': [_I, _I, _I, _I, _P, _L, _P, _P, _P, _L, _P, _L, _P, _L, _P, _P, _P, _L, _P,
                      _L, _P, _L, _P],
    'srnn_gru_cell_bwd': [_I, _I, _I, _P, _L, _P, _L, _P, _P, _P, _P, _L, _P, _L, _P, _L, _P, _L,
                          _P, _L, _P, _P],
    'srnn_mlp_l1': [_I, _P, _P, _L, _I, _I, _I, _I, _P, _L, _P, _L, _I, _I, _I, _P],
    'srnn_mlp_dtab': [_I, _P, _L, _P, _L, _I, _I, _I, _P, _I, _I, _I, _I, _P, _SZ, _P],
    'srnn_mlp_dtab2': [_I, _P, _L, _P, _L, _I, _I, _I, _P, _I, _I, _I, _I, _P, _SZ, _P,
                       ctypes.POINTER(_I), _P],
    'srnn_mlp_dtab3': [_I, _P, _L, _P, _L, _I, _I, _I, _P, _I, _I, _I, _I, _P, _SZ, _P,
                       ctypes.POINTER(_I), _P, _P],
    'srnn_mlp_dtab4': [_I, _P, _L, _P, _L, _I, _I, _I, _P, _I, _I, _I, _I, _P, _SZ, _P,
                       ctypes.POINTER(_I), _P, _P, _P],
    'srnn_gemm_amax_next': [_P],
    'srnn_cast_multi': [_I, _P, _P, _P, _P],
    'srnn_gemm_amax_blk_next': [_P, _P],
    'srnn_gemm_csum_next': [_P],
    'srnn_logsoftmax_nll': [_P, _L, _P, _L, _I, _L, _I, _P, _P, _L, _P, _I, _L, _F, _P],
    'srnn_logsoftmax_bwd': [_P, _L, _P, _L, _L, _I, _P, _I, _L, _P],
    'srnn_nll_fwd': [_P, _L, _P, _L, _I, _L, _P, _P],
    'srnn_nll_bwd': [_P, _L, _I, _L, _I, _P, _L, _F, _P, _P],
    'srnn_weight_norm_fwd': [_P, _P, _P, _P, _I, _L, _P],
    'srnn_weight_norm_bwd': [_P, _P, _P, _P, _P, _I, _L, _I, _P],
    'srnn_permute3': [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    'srnn_copy2d': [_I, _I, _I, _I, _P, _L, _P, _L, _P],
    'srnn_gather_rows': [_P, _L, _P, _L, _I, _P, _I, _L, _P],
    'srnn_scatter_add_rows': [_P, _L, _P, _L, _I, _P, _L, _P],
    'srnn_index_add_rows': [_P, _L, _I, _P, _L, _I, _P, _L, _P],
    'srnn_set_device_share': [_I],
    'srnn_hold_cus': [_I, _I, _P, _P],
    'srnn_axpby': [_P, _P, _P, _F, _F, _L, _P],
    'srnn_add_bcast_rows': [_P, _P, _I, _I, _I, _L, _P],
    'srnn_segsum': [_P, _L, _I, _I, _I, _P, _P],
    'srnn_colsum': [_I, _P, _L, _L, _I, _P, _F, _I, _P, _L, _P],
    'srnn_adam_clip': [_P, _P, _P, _P, _P, _L, _F, _F, _D, _D, _D, _D, _L, _P],
    'srnn_adam_clip_multi': [_I, _P, _P, _P, _P, _P, _P, _F, _F, _D, _D, _D, _D, _L, _P],
    'srnn_gru_seq_fwd': [_I, _I, _I, _I, _P, _L, _L, _P, _P, _P, _P, _P, _P, _L, _L, _P, _L, _L,
                         _P, _SZ, _P],
    'srnn_gru_seq_bwd': [_I, _I, _I, _I, _P, _L, _L, _P, _L, _L, _P, _L, _L, _P, _P, _P, _P, _P,
                         _L, _L, _P, _P, _SZ, _P],
    'srnn_gru_xcd_fwd': [_I, _I, _I, _I, _P, _L, _L, _P, _P, _P, _P, _P, _L, _L, _P, _L, _L, _P,
                         _SZ, _P],
    'srnn_gru_xcd_fwd2': [_I, _I, _I, _I, _P, _L, _L, _P, _P, _P, _P, _P, _L, _L, _P, _L, _L, _P,
                          _P, _SZ, _P],
    'srnn_gru_xcd_bwd': [_I, _I, _I, _I, _P, _L, _L, _P, _L, _L, _P, _L, _L, _P, _P, _P, _P, _P,
                         _L, _L, _P, _P, _SZ, _P],
    'srnn_gru_xcd_bwd2': [_I, _I, _I, _I, _P, _L, _L, _P, _L, _L, _P, _L, _L, _P, _P, _P, _P, _P,
                          _P, _P, _L, _L, _P, _P, _SZ, _P],
    'srnn_weight_norm_scale': [_P, _P, _P, _I, _L, _P],
    'srnn_convt_fold': [_P, _P, _P, _I, _I, _I, _I, _P],
    'srnn_convt_wn_bwd': [_P, _P, _P, _P, _P, _I, _I, _I, _P],
    'srnn_gen_workspace_size': [_P, _I, ctypes.POINTER(_SZ)],
    'srnn_generate': [_P, _I, _I, _P, _P, _P, _U64, _P, _P, _P, _SZ, _I, _P],
    'srnn_generate2': [_P, _I, _I, _P, _P, _P, _U64, _I, _P, _P, _P, _SZ, _I, _P],
    'srnn_persistent_flag_to_f32': [_P, _P],
    'srnn_persistent_flag_or_f32': [_P, _P],
    'srnn_persistent_flag_snapshot': [_P, _P],
    'srnn_persistent_flag_to': [_P, _I, _P],
    'srnn_persistent_flag_or': [_P, _I, _P],
    'srnn_adam_clip_multi2': [_I, _P, _P, _I, _F, _P, _P, _P, _P, _F, _F, _D, _D, _D, _D, _L,
                              _P],
    'srnn_pack_grads': [_I, _P, _P, _P, _P, _I, _P],
    'srnn_adam_clip_multi3': [_I, _P, _P, _I, _F, _P, _P, _P, _P, _F, _F, _D, _D, _D, _D, _L,
                              _P, _P],
    'srnn_step_advance': [_P, _I, _P],
    'srnn_nll_logsoftmax_bwd': [_P, _L, _I, _L, _I, _P, _L, _F, _P, _P, _I, _L, _P],
}


class SrnnTier(ctypes.Structure):
    _fields_ = [('frame_size', _I), ('n_frame_samples', _I), ('in_dim', _I),
                ('w_in', _P), ('b_in', _P),
                ('w_ih', _P * MAX_RNN), ('b_ih', _P * MAX_RNN),
                ('w_hh', _P * MAX_RNN), ('b_hh', _P * MAX_RNN),
                ('w_up', _P), ('b_up', _P), ('h0', _P)]


class SrnnModel(ctypes.Structure):
    _fields_ = [('n_tiers', _I), ('n_rnn', _I), ('dim', _I), ('q_levels', _I),
                ('cond_dim', _I), ('dtype', _I), ('tier', SrnnTier * MAX_TIERS),
                ('tab', _P), ('w_hid', _P), ('b_hid', _P), ('w_out', _P), ('b_out', _P)]


class _Lib:
    def __init__(self, path):
        if not os.path.exists(path):
            raise ImportError('libsamplernn_hip.so not built (%s); run __graft_entry__.build()'
                              % path)
        self.dll = ctypes.CDLL(path)
        self.dll.srnn_last_error.restype = ctypes.c_char_p
        self.dll.srnn_last_error.argtypes = []
        # the library must be built from the sources beside it: a stale .so that still has
        # every symbol would otherwise run old kernels silently
        self.dll.srnn_build_hash.restype = ctypes.c_char_p
        self.dll.srnn_build_hash.argtypes = []
        self.build_hash = self.dll.srnn_build_hash().decode()
        want = csrc_hash()
        if self.build_hash != want and os.environ.get('SRNN_ALLOW_STALE_LIB', '0') != '1':
            raise ImportError('%s is stale: built from sources %s, the tree has %s -- rebuild '
                              '(__graft_entry__.build() or make -C csrc)'
                              % (path, self.build_hash, want))
        for name, args in _SIGS.items():
            fn = getattr(self.dll, name)
            fn.argtypes = args
            fn.restype = _I
        # query entry points called on .dll directly (pointers are passed as plain ints, so
        # every pointer argument needs its declared type)
        for name, args in (('srnn_gru_xcd_error', [_P]), ('srnn_persistent_error_take', []),
                           ('srnn_gemm_amax_taken', []), ('srnn_gemm_csum_taken', []),
                           ('srnn_gemm_logsoftmax_next', []), ('srnn_gemm_logsoftmax_taken', []),
                           ('srnn_blaslt_calls', []), ('srnn_blaslt_set_tune', [_I]),
                           ('srnn_blaslt_set_min', [ctypes.c_longlong, ctypes.c_double])):
            fn = getattr(self.dll, name)
            fn.argtypes = args
            fn.restype = _I

    def call(self, name, *args):
        rc = getattr(self.dll, name)(*args)
        if rc != 0:
            raise RuntimeError('%s failed (%d): %s' % (name, rc,
                                                       self.dll.srnn_last_error().decode()))

    def call_timed(self, name, *args):
        t0 = time.perf_counter()
        try:
            self._call(name, *args)
        finally:
            key = name if name != 'srnn_gemm' else 'gemm %dx%dx%d t%d%d' % (
                args[4], args[5], args[6], args[2], args[3])
            n, s = HOST_TIME.get(key, (0, 0.0))
            HOST_TIME[key] = (n + 1, s + time.perf_counter() - t0)


# SRNN_HOST_PROF=1: host seconds spent inside each C entry point (argument conversion + the
# HIP launch calls), to find launch-bound stretches of a step; bench.py prints the table
HOST_TIME = {}
if os.environ.get('SRNN_HOST_PROF', '0') == '1':
    _Lib._call = _Lib.call
    _Lib.call = _Lib.call_timed


_LIB = None


def lib():
    """The loaded library (raises if absent: no fallback)."""
    global _LIB
    if _LIB is None:
        _LIB = _Lib(LIB_PATH)
    return _LIB


def exported_symbols():
    return sorted(_SIGS) + ['srnn_last_error', 'srnn_abi_version', 'srnn_gru_seq_supported',
                            'srnn_gen_persistent_rows', 'srnn_gru_xcd_work_bytes',
                            'srnn_gru_xcd_bwd_work_bytes', 'srnn_gru_xcd_error',
                            'srnn_persistent_error_take', 'srnn_gemm_amax_taken',
                            'srnn_gemm_csum_taken', 'srnn_blaslt_calls', 'srnn_device_share',
                            'srnn_build_hash', 'srnn_dtab_packed_ok', 'srnn_gemm_logsoftmax_next',
                            'srnn_gemm_logsoftmax_taken', 'srnn_blaslt_set_min',
                            'srnn_blaslt_set_tune']


# Callbacks run just before a persistent sweep (gru_xcd / gru_seq) is enqueued.  Such a sweep
# needs every workgroup co-resident (one per CU, up to the whole register file), so it must
# not share the GPU with RCCL kernels: partially resident, a sweep and an all-reduce could
# wait on each other across ranks.  distributed.GradAllReduce registers a callback that makes
# the current stream wait for every gradient all-reduce already in flight.
BEFORE_PERSISTENT = []
# ... and AFTER_PERSISTENT right after a sweep is enqueued: GradAllReduce launches the
# all-reduces of buckets that became ready before the sweep here, so their RCCL kernels are
# ordered after it (they overlap the GEMMs that follow) instead of in front of it, where the
# next sweep's fence would wait for them.
AFTER_PERSISTENT = []

# Measurement hook (bench.py): when a dict, the step's heaviest launch sites (the GRU sweeps,
# the dTab scatter, the MLP hidden-layer GEMM, the fused clip+Adam, ...) are bracketed by HIP
# events on the stream they launch on, and site -> [(start, end, work)] collects them, so
# their durations are measured inside the timed TBPTT steps (work = the launch's algorithmic
# flop or bytes)
ROOF_EVENTS = None


def roof_begin():
    """Start event of a probed launch site (None when probing is off)."""
    if ROOF_EVENTS is None:
        return None
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def roof_end(site, ev0, work):
    if ev0 is None or ROOF_EVENTS is None:
        return
    ev1 = torch.cuda.Event(enable_timing=True)
    ev1.record()
    ROOF_EVENTS.setdefault(site, []).append((ev0, ev1, float(work)))


def _run_hooks(lst):
    """Run the registered callbacks (plain callables or weakref.WeakMethod references, whose
    dead entries -- a GradAllReduce that is gone -- are dropped)."""
    dead = []
    for f in lst:
        if isinstance(f, weakref.WeakMethod):
            m = f()
            if m is None:
                dead.append(f)
                continue
            m()
        else:
            f()
    for f in dead:
        lst.remove(f)


def before_persistent_sweep():
    _run_hooks(BEFORE_PERSISTENT)


def after_persistent_sweep():
    _run_hooks(AFTER_PERSISTENT)


def check_persistent_errors():
    """Raise if a persistent GRU sweep gave up a hand-off since the last check (its outputs
    are invalid; the fused clip+Adam already skipped that step's update on the device).
    Synchronises the device; the Trainer calls it once per iteration."""
    fn = lib().dll.srnn_persistent_error_take
    fn.restype = ctypes.c_int
    fn.argtypes = []
    v = fn()
    if v == 2:
        raise RuntimeError('persistent GRU sweep: its workgroups were not all resident within '
                           '30 s (another process holds the CUs; see set_device_share) -- results '
                           'of this step are invalid')
    if v:
        raise RuntimeError('persistent GRU sweep gave up a hand-off (bounded spin) -- results of '
                           'this step are invalid' if v > 0 else
                           'srnn_persistent_error_take: HIP error')


def set_device_share(n):
    """Declare that n processes run persistent kernels on this process's GPU at once (a
    multi-rank rehearsal on one GPU; 1 normally).  Persistent sweeps and the generation loop
    then only take launch shapes whose grids fit the device n times over (their co-residency
    guarantee, csrc/handoff.hpp), chaining smaller launches or taking the per-step kernels
    otherwise.  Call before the first model step (the support predicates are cached)."""
    lib().call('srnn_set_device_share', int(n))
    _GRU_XCD.clear()
    _GRU_SEQ.clear()


class PersistentErrorWatch:
    """Lagged, synchronisation-free form of check_persistent_errors for the training loop
    (trainer/__init__.py:116-117 checks once per iteration): after step n is enqueued a 4-byte
    stream-ordered copy of the sticky flag goes to pinned host memory, and the copy of step
    n - 1 is read -- waiting only on that copy's event, which the GPU has normally passed
    while it runs step n.  The flag is sticky, so a failure in step n - 1 also made step n's
    fused clip+Adam skip its update: `step()` then reports 2 skipped steps (the caller rolls
    the Adam step counters back, optim.py) and raises.  flush() checks the last step with a
    synchronisation (epoch end)."""

    def __init__(self):
        self._bufs = [torch.zeros(1, dtype=torch.int32).pin_memory() for _ in range(2)]
        self._events = [None, None]
        self._n = 0

    def _snapshot(self):
        slot = self._n % 2
        lib().call('srnn_persistent_flag_snapshot', ptr(self._bufs[slot]), stream())
        ev = torch.cuda.Event()
        ev.record()
        self._events[slot] = ev
        self._n += 1

    def _read(self, slot):
        ev = self._events[slot]
        if ev is None:
            return 0
        ev.synchronize()
        self._events[slot] = None
        return int(self._bufs[slot][0])

    def step(self, on_skip=None):
        """Call once per enqueued training step."""
        self._snapshot()
        if self._n >= 2 and self._read((self._n - 2) % 2):
            self._fail(on_skip, 2)

    def flush(self, on_skip=None):
        if self._n and self._read((self._n - 1) % 2):
            self._fail(on_skip, 1)

    def _fail(self, on_skip, skipped):
        for s in range(2):
            self._events[s] = None
        if on_skip is not None:
            on_skip(skipped)
        check_persistent_errors()       # synchronises, clears the flag and raises


_GRU_XCD = {}


def gru_xcd_work_bytes(dtype, B, D):
    """Work-buffer bytes of the XCD-grouped persistent GRU forward (gru_xcd.hip) for (B, D),
    0 when it does not apply (SRNN_GRU_XCD=0 disables it)."""
    if os.environ.get('SRNN_GRU_XCD', '1') == '0':
        return 0
    key = (dtype, B, D)
    if key not in _GRU_XCD:
        fn = lib().dll.srnn_gru_xcd_work_bytes
        fn.argtypes = [_I, _I, _I]
        fn.restype = _SZ
        _GRU_XCD[key] = int(fn(dcode(dtype), B, D))
    return _GRU_XCD[key]


def gru_xcd_bwd_work_bytes(dtype, B, D):
    """Work-buffer bytes of the XCD-grouped persistent GRU backward, 0 when it does not
    apply (SRNN_GRU_XCD=0 disables it)."""
    if os.environ.get('SRNN_GRU_XCD', '1') == '0':
        return 0
    key = ('bwd', dtype, B, D)
    if key not in _GRU_XCD:
        fn = lib().dll.srnn_gru_xcd_bwd_work_bytes
        fn.argtypes = [_I, _I, _I]
        fn.restype = _SZ
        _GRU_XCD[key] = int(fn(dcode(dtype), B, D))
    return _GRU_XCD[key]


def gen_persistent_rows(dtype, n_seqs, dim, fs0, q_levels=256):
    """Rows per group of the persistent generation loop for this shape (0: per-sample
    kernels)."""
    fn = lib().dll.srnn_gen_persistent_rows
    fn.argtypes = [_I, _I, _I, _I, _I]
    fn.restype = _I
    return int(fn(dcode(dtype), n_seqs, dim, fs0, q_levels))


_GRU_SEQ = {}


def gru_seq_supported(dtype, B, D):
    """Whether the persistent whole-sequence GRU kernel can run (B, D) here (queried once;
    SRNN_GRU_SEQ=0 disables it)."""
    if os.environ.get('SRNN_GRU_SEQ', '1') == '0':
        return False
    key = (dtype, B, D)
    if key not in _GRU_SEQ:
        fn = lib().dll.srnn_gru_seq_supported
        fn.argtypes = [_I, _I, _I]
        fn.restype = _I
        _GRU_SEQ[key] = bool(fn(dcode(dtype), B, D))
    return _GRU_SEQ[key]


# ------------------------------------------------------------------ helpers
def csrc_hash():
    """Content hash of the HIP sources the library is built from (csrc/*.hip, *.hpp, *.h,
    *.cpp and the C-ABI header): 16 hex digits (csrc/srchash.py, which the Makefile also
    compiles into the library as srnn_build_hash()).  Profiles record it, so a committed
    counter pass is only attributed to the kernels it measured (bench.py's roofline.traffic),
    and lib() refuses a library built from other sources."""
    import importlib.util
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location('_srnn_srchash',
                                                  os.path.join(here, 'csrc', 'srchash.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.csrc_hash(os.path.join(here, 'csrc'))


def ptr(t):
    """Device/host pointer of a tensor (None -> NULL).  A plain int: ctypes converts it for
    c_void_p arguments and struct fields without building an object per call."""
    if t is None:
        return None
    return t.data_ptr()


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_dev = torch._C._cuda_getDevice


def stream():
    """hipStream_t of the current torch stream, as an int (hundreds of calls per TBPTT step:
    no torch.cuda.Stream object is built per call)."""
    return _raw_stream(_cur_dev())


def dcode(t_or_dtype):
    dt = t_or_dtype.dtype if isinstance(t_or_dtype, torch.Tensor) else t_or_dtype
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise TypeError('unsupported dtype %s' % dt)


def need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('samplernn_hip: device tensor expected (got %s); the HIP path has '
                               'no CPU fallback' % t.device)


_GEMM_LOG = os.environ.get('SRNN_GEMM_LOG', '0') == '1'


def relu_bits(rows, cols, device):
    """An (rows, ceil(cols / 16)) int16 buffer for a ReLU mask as bits (srnn_gemm_bits)."""
    return torch.empty((rows, (cols + 15) // 16), device=device, dtype=torch.int16)


def relu_bits_grouped(rows, cols, device):
    """A ReLU mask as bits in the grouped layout (u16 [cols / 16][rows], cols % 64 == 0;
    srnn_relu_bits with ldb = 0): a 1-D int16 buffer, passed with row stride 0."""
    if cols % 64:
        raise ValueError('grouped mask bits need cols % 64 == 0 (got %d)' % cols)
    return torch.empty((rows * (cols // 16),), device=device, dtype=torch.int16)


def bits_ld(bits):
    """Row stride (u16) of a bit-mask buffer: 0 for the grouped (1-D) layout."""
    return bits.stride(0) if bits.dim() == 2 else 0


def gemm(a, b, transA=False, transB=False, out=None, out_dtype=torch.float32, bias=None,
         bias_mode=1, relu=False, alpha=1.0, beta=0.0, cin=None, mask=None, M=None, N=None, K=None,
         lda=None, ldb=None, ldc=None, ldcin=None, batch=1, sA=0, sB=0, sC=0, sCin=0, tile=-1,
         mask_bits=None, bits_out=None):
    """C = act(alpha op(A) op(B) + beta Cin + bias) on row-major 2-D views (or strided batches).
    mask_bits / bits_out: the ReLU mask as bits (relu_bits buffers), read in place of `mask` /
    written for C (batch 1)."""
    need_cuda(a, b)
    if M is None:
        M = a.shape[1] if transA else a.shape[0]
        K = a.shape[0] if transA else a.shape[1]
        N = b.shape[0] if transB else b.shape[1]
    if lda is None:
        lda = a.stride(0)
    if ldb is None:
        ldb = b.stride(0)
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=out_dtype)
    if ldc is None:
        ldc = out.stride(0) if out.dim() > 1 else N
    if cin is not None and ldcin is None:
        ldcin = cin.stride(0)
    if a.dtype != b.dtype:
        raise TypeError('gemm operands must share a dtype (%s vs %s)' % (a.dtype, b.dtype))
    if _GEMM_LOG:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    if mask_bits is not None or bits_out is not None:
        if batch != 1 or mask is not None:
            raise ValueError('gemm: bit masks need batch 1 and no tensor mask')
        lib().call('srnn_gemm_bits', dcode(a), dcode(out), int(transA), int(transB), M, N, K,
                   alpha, ptr(a), lda, ptr(b), ldb, beta, ptr(cin), ldcin or 0, ptr(out), ldc,
                   ptr(bias), bias_mode, int(relu), tile, ptr(mask_bits),
                   bits_ld(mask_bits) if mask_bits is not None else 0, ptr(bits_out),
                   bits_ld(bits_out) if bits_out is not None else 0, stream())
    else:
        lib().call('srnn_gemm', dcode(a), dcode(out), int(transA), int(transB), M, N, K, alpha,
                   ptr(a), lda, sA, ptr(b), ldb, sB, beta, ptr(cin), ldcin or 0, sCin, ptr(out),
                   ldc, sC, ptr(bias), bias_mode, int(relu), batch, tile, ptr(mask),
                   (mask.stride(0) if mask is not None else 0), stream())
    if _GEMM_LOG:
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6
        sys.stderr.write('gemm M=%d N=%d K=%d batch=%d tA=%d tB=%d %s->%s mask=%d bias=%d relu=%d '
                         'cin=%d %.1f us %.1f TF/s\n' % (
                             M, N, K, batch, transA, transB, a.dtype, out.dtype, mask is not None,
                             bias is not None, relu, cin is not None, us,
                             2.0 * M * N * K * batch / us / 1e6))
    return out


def linear(x, w, bias=None, relu=False, out_dtype=torch.float32, out=None, cin=None, beta=0.0,
           bits_out=None):
    """y = act(x . w^T + bias (+ beta * cin)) for 2-D x (M, K) and w (N, K)."""
    return gemm(x, w, transB=True, bias=bias, relu=relu, out_dtype=out_dtype, out=out, cin=cin,
                beta=beta, bits_out=bits_out)


def colsum(x, rows, cols, lds=None, out=None, alpha=1.0, accumulate=False):
    need_cuda(x)
    if out is None:
        out = torch.empty(cols, device=x.device, dtype=torch.float32)
    lds = cols if lds is None else lds
    # the first pass writes at most ~2048 / ceil(cols / 64) partial rows
    nrb = max(1, min((rows + 63) // 64, 2048 // max(1, (cols + 63) // 64)))
    work = torch.empty(nrb * cols + 256, device=x.device, dtype=torch.float32)
    lib().call('srnn_colsum', dcode(x), ptr(x), lds, rows, cols, ptr(out), alpha, int(accumulate),
               ptr(work), work.numel(), stream())
    return out


def cast(x, dtype):
    """Dtype conversion through the HIP copy kernel (contiguous 2-D view)."""
    need_cuda(x)
    if x.dtype == dtype:
        return x
    x = x.contiguous()
    out = torch.empty(x.shape, device=x.device, dtype=dtype)
    cols = x.shape[-1] if x.dim() > 0 else 1
    rows = x.numel() // max(cols, 1)
    lib().call('srnn_copy2d', dcode(x), dcode(out), rows, cols, ptr(x), cols, ptr(out), cols,
               stream())
    return out


# Compute-dtype (bf16) copies of parameters, kept across steps: id(param) -> (weakref, copy,
# data_ptr, _version).  A copy is valid while the parameter's storage and version are
# unchanged; torch in-place updates (load_state_dict, manual edits) bump the version, and the
# fused clip+Adam (optim.py), which writes the parameter through a raw pointer, rewrites the
# copy in the same kernel (srnn_adam_clip_multi's p_bf16), so the copy stays valid.
_SHADOW = {}


def cast_param(p, dtype):
    """`p` (an fp32 parameter) in `dtype`: the cached copy when still valid, else a fresh cast
    that becomes the cached copy."""
    if p.dtype == dtype:
        return p
    key = id(p)
    e = _SHADOW.get(key)
    if e is not None and e[0]() is p and e[1].dtype == dtype and e[2] == p.data_ptr() and \
            e[3] == p._version:
        return e[1]
    c = cast(p.detach(), dtype)
    if e is None or e[0]() is not p:
        # evict the copy with its parameter (no bf16 copies of dead parameters stay allocated)
        weakref.finalize(p, _SHADOW.pop, key, None)
    _SHADOW[key] = (weakref.ref(p), c, p.data_ptr(), p._version)
    return c


def shadow_refreshed(p):
    """The fused clip+Adam (srnn::adam_clip_, which declares its in-place writes and so bumps
    the parameter's version counter) rewrote p and its bf16 copy together: keep the copy valid
    at p's new version."""
    e = _SHADOW.get(id(p))
    if e is not None and e[0]() is p and e[2] == p.data_ptr():
        _SHADOW[id(p)] = (e[0], e[1], p.data_ptr(), p._version)


def shadow_of(p):
    """The valid bf16 copy of parameter p, or None (the fused Adam step refreshes it)."""
    e = _SHADOW.get(id(p))
    if e is not None and e[0]() is p and e[2] == p.data_ptr() and e[3] == p._version and \
            e[1].dtype == torch.bfloat16:
        return e[1]
    return None


def permute3(src, perm, dtype=torch.float32, out=None, accumulate=False):
    """out = src.permute(perm).contiguous() (src fp32, 3-D) via the HIP permute kernel."""
    need_cuda(src)
    src = src.contiguous()
    d = list(src.shape)
    if out is None:
        out = torch.empty([d[p] for p in perm], device=src.device, dtype=dtype)
    lib().call('srnn_permute3', ptr(src), ptr(out), dcode(out), d[0], d[1], d[2], perm[0], perm[1],
               perm[2], int(accumulate), stream())
    return out


def weight_norm(g, v):
    """w = g * v / ||v|| (torch weight_norm, dim=0)."""
    need_cuda(g, v)
    v = v.contiguous()
    w = torch.empty_like(v)
    O = v.shape[0]
    lib().call('srnn_weight_norm_fwd', ptr(g), ptr(v), ptr(w), None, O, v.numel() // O, stream())
    return w


def convt_operand(g, v, k, dtype):
    """The upsampling GEMM operand W_up (k, Cout, Cin) = (g * v / ||v||).permute(2, 1, 0) in
    `dtype`, straight from v (conv_t weight (Cin, Cout, k)); g None = no weight norm."""
    need_cuda(v)
    v = v.contiguous()
    Cin, Cout = v.shape[0], v.shape[1]
    out = torch.empty((k, Cout, Cin), device=v.device, dtype=dtype)
    scale = None
    if g is not None:
        scale = torch.empty(Cin, device=v.device, dtype=torch.float32)
        lib().call('srnn_weight_norm_scale', ptr(g), ptr(v), ptr(scale), Cin, v.numel() // Cin,
                   stream())
    lib().call('srnn_convt_fold', ptr(v), ptr(scale), ptr(out), dcode(out), Cin, Cout, k, stream())
    return out


def convt_operand_ok(Cin, Cout, k):
    return Cin % 64 == 0 and (Cout * k) % 64 == 0 and 64 % k == 0


def convt_wn_bwd(g, v, dwt, k):
    """(dg, dv) of the weight norm from the transposed GEMM gradient dwt (Cin, k * Cout),
    rows [i][j * Cout + o]."""
    v = v.contiguous()
    Cin, Cout = v.shape[0], v.shape[1]
    dg = torch.empty_like(g)
    dv = torch.empty_like(v)
    lib().call('srnn_convt_wn_bwd', ptr(g), ptr(v), ptr(dwt.contiguous()), ptr(dg), ptr(dv), Cin,
               Cout, k, stream())
    return dg, dv


def weight_norm_bwd(g, v, dw):
    v = v.contiguous()
    dw = dw.contiguous()
    O = v.shape[0]
    dg = torch.empty_like(g)
    dv = torch.empty_like(v)
    lib().call('srnn_weight_norm_bwd', ptr(g), ptr(v), ptr(dw), ptr(dg), ptr(dv), O,
               v.numel() // O, 0, stream())
    return dg, dv
