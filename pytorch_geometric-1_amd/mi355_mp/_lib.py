"""ctypes binding of the C-ABI in include/mi355_mp.h (libmi355_mp.so).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C pytorch_geometric-1_amd/csrc``).  There is no fallback: if the
library is missing, or a tensor is not on a ROCm device, every op raises.
Only plain pointers, sizes and the HIP stream handle cross the boundary.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB_PATH = os.path.join(_HERE, "libmi355_mp.so")
LIB_PATH = os.environ.get("MI355_MP_LIB", DEFAULT_LIB_PATH)

MP_OK = 0
MP_REDUCE = {"sum": 0, "add": 0, "mean": 1, "max": 2, "min": 3}
MP_FLAG_INIT_FROM_OUT = 1
MP_FLAG_PYG_MASK = 2
MP_FLAG_SKIP_EMPTY = 4
MP_STAGE_MAIN = 1
MP_STAGE_FIXUP = 2
MP_STAGE_STATS = 4
MP_STAGE_ALL = 7
MP_TUNE_FLAT_VEC1_MIN_BYTES = 1
MP_TUNE_FLAT_SMEM = 2
MP_TUNE_FLAT_MIN_F = 3
MP_TUNE_FLAT_MIN_F_ARG = 4
MP_TUNE_FLAT_NARROW_VEC1 = 5
MP_TUNE_FLAT_VEC = 6
MP_TUNE_FLAT_VEC_ARG = 7
MP_TUNE_FLAT_SEQ_TILES = 8
MP_TUNE_FLAT_FAR_MIN_BYTES = 9
MP_TUNE_GAT_BWD_VEC = 10
MP_DTYPE = {torch.float32: 0, torch.float64: 1, torch.float16: 2, torch.bfloat16: 3, torch.int64: 4}
MP_LOOPS_REMOVE = 0
MP_LOOPS_ADD = 1
MP_LOOPS_ADD_REMAINING = 2

c_p = ctypes.c_void_p
i64 = ctypes.c_int64
u64 = ctypes.c_uint64
i32 = ctypes.c_int32
f32 = ctypes.c_float
sz = ctypes.c_size_t


class MpCsr(ctypes.Structure):
    _fields_ = [
        ("rowptr", c_p), ("col", c_p), ("eid", c_p), ("wave_row", c_p),
        ("wave_slot", c_p), ("split_waves", c_p), ("n_rows", i64),
        ("n_edges", i64), ("chunk", i32), ("n_waves", i32), ("n_split", i32),
        ("n_cols", i32), ("n_ids", i64),
    ]


# name -> (restype, argtypes); mirrors include/mi355_mp.h one to one.
SIGNATURES = {
    "mp_last_error": (ctypes.c_char_p, []),
    "mp_abi_version": (ctypes.c_int, []),
    "mp_source_hash": (ctypes.c_char_p, []),
    "mp_tune": (i64, [i32, i64]),
    "mp_csr_build_workspace": (sz, [i64, i64]),
    "mp_csr_build": (ctypes.c_int, [c_p, c_p, i64, i64, i64, c_p, c_p, c_p, c_p, c_p, sz, c_p]),
    "mp_schedule_n_waves": (i32, [i64, i64, i32]),
    "mp_schedule_workspace": (sz, [i32]),
    "mp_schedule_build": (ctypes.c_int, [c_p, i64, i64, i32, i32, c_p, c_p, c_p, c_p, c_p, sz, c_p]),
    "mp_aggregate_slab_bytes": (sz, [ctypes.POINTER(MpCsr), i32, i32]),
    "mp_aggregate_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, i64, i32, i32, i32, c_p,
                                        c_p, i64, c_p, c_p, sz, i32, c_p]),
    "mp_aggregate_kernel_name": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, i64, i32, i32, c_p, c_p, i64,
                                                ctypes.c_char_p, sz, c_p]),
    "mp_gat_node_scores_f32": (ctypes.c_int, [c_p, i64, i32, i32, c_p, c_p, c_p, c_p]),
    "mp_gat_slab_bytes": (sz, [ctypes.POINTER(MpCsr), i32, i32]),
    "mp_gat_aggregate_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, c_p, i32, i32, f32, c_p,
                                            c_p, i64, c_p, c_p, sz, i32, c_p]),
    "mp_gat_aggregate_att_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, c_p, c_p, i32, i32, f32, c_p,
                                                c_p, i64, c_p, c_p, sz, i32, c_p]),
    "mp_gat_forward_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, i32, i32, f32, c_p, c_p, i64, c_p, c_p,
                                          c_p, c_p, sz, i32, c_p]),
    "mp_gat_forward_train_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, i32, i32, f32, c_p, c_p, i64, c_p,
                                                c_p, c_p, c_p, c_p, c_p, c_p, sz, i32, c_p]),
    "mp_gat_train_ok": (ctypes.c_int, [i32, i32]),
    "mp_gat_train_slab_bytes": (sz, [ctypes.POINTER(MpCsr), i32, i32]),
    "mp_gat_aggregate_train_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, c_p, c_p, i32, i32, f32,
                                                  c_p, c_p, i64, c_p, c_p, c_p, c_p, c_p, sz, i32, c_p]),
    "mp_gat_two_pass_ok": (ctypes.c_int, [i32, i32]),
    "mp_gat_softmax_aggregate_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, c_p, c_p, i32, i32, f32,
                                                    c_p, c_p, i64, c_p, c_p, sz, i32, c_p]),
    "mp_gat_alpha_f32": (ctypes.c_int, [c_p, c_p, i64, i32, c_p, c_p, f32, c_p, c_p, c_p]),
    "mp_csr_slot_rows": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p]),
    "mp_gat_alpha_csr_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, c_p, i32, f32, c_p, c_p, c_p,
                                            c_p]),
    "mp_aggregate_heads_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, i32, c_p, i64, i32, c_p, i64, c_p,
                                              sz, i32, c_p]),
    "mp_gat_sddmm_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, i64, c_p, i64, i32, i32, c_p, c_p]),
    "mp_gat_backward_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, i64, c_p, c_p, c_p, c_p, i32, i32,
                                           ctypes.c_float, c_p, c_p, c_p, sz, c_p, sz, i32, c_p]),
    "mp_gat_backward_train_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, i64, c_p, c_p, c_p, c_p, i32, i32,
                                                 ctypes.c_float, c_p, c_p, c_p, c_p, sz, i32, c_p]),
    "mp_gat_aggregate_train_drop_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, c_p, c_p, i32, i32, f32,
                                                       c_p, c_p, i64, c_p, c_p, c_p, c_p, u64, f32, c_p, c_p, sz, i32,
                                                       c_p]),
    "mp_gat_backward_train_drop_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, i64, c_p, c_p, c_p, c_p, i32,
                                                      i32, f32, c_p, u64, f32, c_p, c_p, c_p, c_p, sz, i32, c_p]),
    "mp_gat_dropout_keep": (ctypes.c_int, [u64, f32, i32, i64, c_p, c_p, c_p]),
    "mp_gat_wide_ok": (ctypes.c_int, [i32, i32]),
    "mp_gat_node_scores_wide_f32": (ctypes.c_int, [c_p, i64, i32, i32, c_p, c_p, c_p, c_p]),
    "mp_gat_backward_prep_wide_f32": (ctypes.c_int, [c_p, i64, c_p, i64, c_p, c_p, c_p, c_p, c_p, i64, i32, i32, c_p,
                                                     sz, c_p, c_p]),
    "mp_gat_backward_wide_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, i64, c_p, c_p, i32, i32, f32, u64, f32, c_p,
                                                c_p, c_p, sz, c_p, sz, c_p, sz, i32, c_p]),
    "mp_gat_backward_epilogue_wide_f32": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, c_p, i64, i32, i32, c_p]),
    "mp_segment_offset_i64": (ctypes.c_int, [c_p, i64, i32, i64, c_p, c_p, i64, c_p]),
    "mp_segment_ids_i64": (ctypes.c_int, [c_p, i64, c_p, i64, c_p]),
    "mp_gat_backward_prep_f32": (ctypes.c_int, [c_p, i64, c_p, i64, c_p, c_p, c_p, i64, i32, i32, c_p, sz, c_p, sz,
                                                c_p]),
    "mp_gat_backward_prep_train_f32": (ctypes.c_int, [c_p, i64, c_p, i64, c_p, c_p, c_p, c_p, c_p, i64, i32, i32,
                                                      c_p, sz, c_p, sz, c_p, c_p]),
    "mp_gat_bwd_blocks": (ctypes.c_int, [i64]),
    "mp_col_sums_f32": (ctypes.c_int, [c_p, i64, i64, i32, c_p, sz, c_p]),
    "mp_gemm_rows_f32": (ctypes.c_int, [c_p, i64, i64, i32, c_p, i32, i32, c_p, i64, i32, c_p]),
    "mp_gat_backward_finish_f32": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, i64, i32, i32, c_p, sz, c_p]),
    "mp_gat_merge_partials_f32": (ctypes.c_int, [i64, i32, i32, c_p, c_p, i64, c_p, sz, i64, c_p, sz, c_p, c_p, i64,
                                                 c_p, c_p, c_p, c_p]),
    "mp_aggregate_tiles_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p, i64, i32, i64, i32, i32, i32, c_p,
                                              c_p, c_p, i64, i32, i64, c_p, sz, i32, c_p]),
    "mp_heads_outer_add_f32": (ctypes.c_int, [c_p, i64, c_p, i64, i32, i32, c_p, i64, c_p]),
    "mp_gather_rows_f32": (ctypes.c_int, [c_p, i64, c_p, i64, i32, c_p, i64, c_p]),
    "mp_permute_f32": (ctypes.c_int, [c_p, c_p, i64, c_p, c_p]),
    "mp_scatter_arg_backward_f32": (ctypes.c_int, [c_p, c_p, i64, i32, i64, c_p, i64, c_p]),
    "mp_self_loop_count": (ctypes.c_int, [c_p, c_p, i64, i64, c_p, c_p]),
    "mp_self_loops_workspace": (sz, [i64, i64]),
    "mp_self_loops": (ctypes.c_int, [c_p, c_p, i64, i64, i32, i64, c_p, c_p, c_p, c_p, sz, c_p]),
    "mp_gather_fill_f32": (ctypes.c_int, [c_p, c_p, i64, f32, c_p, c_p]),
    "mp_shard_plan_workspace": (sz, [i64, i64]),
    "mp_shard_plan": (ctypes.c_int, [c_p, c_p, i64, i64, c_p, i32, i32, i64, i64, c_p, c_p, c_p, c_p, c_p, c_p, sz,
                                     c_p]),
    "mp_gcn_norm_f32": (ctypes.c_int, [c_p, c_p, c_p, i64, i64, c_p, c_p, c_p]),
    "mp_gcn_norm_from_deg_f32": (ctypes.c_int, [c_p, c_p, c_p, i64, i64, c_p, c_p, c_p]),
    "mp_segment_sum_serial_f32": (ctypes.c_int, [c_p, c_p, c_p, i64, c_p, c_p]),
    "mp_csr_inverse_eid": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, c_p]),
    "mp_arg_mask_words": (i32, [i32]),
    "mp_arg_winner_mask": (ctypes.c_int, [c_p, i64, i32, i64, c_p, c_p, sz, c_p]),
    "mp_scatter_arg_backward_csr_f32": (ctypes.c_int, [ctypes.POINTER(MpCsr), c_p, sz, c_p, i64, i32, c_p, c_p, i64,
                                                       c_p]),
    "mp_scatter_arg_grad_w_f32": (ctypes.c_int, [c_p, c_p, i64, c_p, c_p, sz, i32, c_p, i64, c_p, i64, c_p, c_p]),
    "mp_segment_reduce": (ctypes.c_int, [ctypes.POINTER(MpCsr), i32, c_p, i64, i32, i32, i32, c_p, i64, c_p, c_p]),
    "mp_gather_rows_any": (ctypes.c_int, [i32, c_p, i64, c_p, i64, i32, c_p, i64, c_p]),
    "mp_scatter_arg_any": (ctypes.c_int, [i32, c_p, c_p, i64, i32, i64, c_p, i64, c_p]),
}

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


class NativeLibraryStale(RuntimeError):
    pass


# the C-ABI version these bindings are written for (include/mi355_mp.h MP_ABI_VERSION)
ABI_VERSION = 7


def load(path=None):
    """Load (once) and return the native library; raise if it is absent, or
    (the in-tree library) if it was built from other sources than the ones
    beside it -- the library carries its source hash (mp_source_hash)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NativeLibraryMissing(
            "mi355_mp: native library %s not found; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback)" % p)
    if path is None and os.path.abspath(p) == os.path.abspath(DEFAULT_LIB_PATH):
        built = library_hash(p)
        want = source_hash()
        if built != want:
            raise NativeLibraryStale(
                "mi355_mp: %s was built from sources %s, the tree holds %s; rebuild it with "
                "`python -c 'import __graft_entry__ as g; g.build()'`" % (p, built, want))
    # RTLD_LOCAL: every build keeps its own kernels.  With RTLD_GLOBAL a second build
    # loaded into the process (an A/B variant) binds its template kernel stubs to the
    # first build's same-named definitions and silently runs the first build's code.
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mp_abi_version() != ABI_VERSION:
        raise NativeLibraryStale("mi355_mp: %s has C-ABI %d, these bindings need %d" % (p, lib.mp_abi_version(),
                                                                                       ABI_VERSION))
    if path is None:
        _lib = lib
    return lib


def library_hash(path=None):
    """The source hash compiled into a library file (mp_source_hash); needs no
    GPU.  'unknown' for a library built without it."""
    lib = ctypes.CDLL(path or LIB_PATH, mode=ctypes.RTLD_LOCAL)
    try:
        fn = lib.mp_source_hash
    except AttributeError:
        return "unknown"
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    return fn().decode()


def source_hash():
    """sha256 over the native sources the library is built from (csrc/*.hip,
    csrc/*.h, csrc/*.cpp, csrc/Makefile, include/mi355_mp.h); the Makefile
    compiles the same hash into the library.  Profile summaries record it, so a
    committed counter profile is only used for the build it measured."""
    import glob
    import hashlib
    csrc = os.path.join(os.path.dirname(_HERE), "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))
                   + glob.glob(os.path.join(csrc, "*.cpp")))
    files += [os.path.join(csrc, "Makefile"),
              os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "mi355_mp.h")]
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def kernel_name(csr_struct, w, x, ldx, F, reduce, bias, out, ldo, device=None):
    """Demangled name of the main kernel mp_aggregate_f32 dispatches for these
    arguments (mp_aggregate_kernel_name)."""
    buf = ctypes.create_string_buffer(1024)
    check(load().mp_aggregate_kernel_name(csr_struct, w, x, ldx, F, MP_REDUCE[reduce], bias, out, ldo, buf, 1024,
                                          stream_ptr(device)), "mp_aggregate_kernel_name")
    return buf.value.decode()


def check(rc, what):
    if rc != MP_OK:
        msg = load().mp_last_error().decode(errors="replace")
        raise RuntimeError("%s failed (code %d): %s" % (what, rc, msg))


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def nbytes(t):
    """Extent in bytes of a caller-allocated array passed to the C-ABI (ABI 6:
    workspaces and partial arrays travel with their size; 0 for None)."""
    return 0 if t is None else t.numel() * t.element_size()


def require_device(*tensors):
    """Every hot-path op runs on the GPU only; there is no CPU fallback."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "mi355_mp: tensors must be on a ROCm (cuda) device; got %s. "
                "The MI355X engine has no CPU fallback." % t.device)
