"""Standalone check + timing of tools/dbg/gemm_mfma.hip (k_gemm_n256) against torch.matmul
(hipBLASLt) for the configs' x @ W and g @ W^T shapes.  Build:
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Iinclude \\
    -Ipytorch_geometric-1_amd/csrc tools/dbg/gemm_mfma.hip \\
    tools/dbg/gemm_probe_stub.cpp -o tools/dbg/_gemm_probe.so"""
import ctypes, json, os
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_gemm_probe.so"))
f = lib.mp_gemm_n256_f32
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
              ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
dev = "cuda"
torch.manual_seed(0)


def gemm(a, w, trans):
    c = torch.empty(a.shape[0], 256, device=dev)
    rc = f(a.data_ptr(), a.stride(0), a.shape[0], 256, w.data_ptr(), int(trans), 256, c.data_ptr(), c.stride(0),
           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    return c


def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {}
w = torch.randn(256, 256, device=dev) * 0.06
for M in (1, 63, 64, 65, 1000, 4097, 100003):
    x = torch.randn(M, 256, device=dev)
    for trans in (0, 1):
        ref = (x.double() @ (w.double().t() if trans else w.double()))
        c = gemm(x, w, trans)
        err = ((c.double() - ref).abs() / (ref.abs() + 1.0)).max().item()
        tw = torch.matmul(x, w.t() if trans else w)
        res["M%d_t%d" % (M, trans)] = {"max_rel_err_vs_fp64": err,
                                       "max_abs_vs_torch": (c - tw).abs().max().item()}
        # the MFMA's k-ordered chain == a sequential fmaf loop from 0, on a few rows
        rows = x[: min(M, 3)].double().cpu()
        wd = (w.t() if trans else w).double().cpu()
        import numpy as np
        xs = x[: min(M, 3)].cpu().numpy(); ws = (w.t() if trans else w).contiguous().cpu().numpy()
        seq = np.zeros((xs.shape[0], 256), dtype=np.float32)
        for k in range(256):
            seq = (seq.astype(np.float64) + xs[:, k:k + 1].astype(np.float64) * ws[k:k + 1, :].astype(np.float64)).astype(np.float32)
        res["M%d_t%d" % (M, trans)]["rows_eq_seq_fma"] = bool(np.array_equal(seq, c[: xs.shape[0]].cpu().numpy()))
# a strided A (lda = 260) and ldc = 264
xa = torch.randn(5000, 260, device=dev)[:, :256]
cfull = torch.zeros(5000, 264, device=dev)
rc = f(xa.data_ptr(), 260, 5000, 256, w.data_ptr(), 0, 256, cfull.data_ptr(), 264,
       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
res["strided"] = {"rc": rc, "err": (cfull[:, :256] - xa @ w).abs().max().item(),
                  "pad_untouched": bool((cfull[:, 256:] == 0).all().item())}
M = 1 << 21
x = torch.randn(M, 256, device=dev)
g = torch.randn(M, 256, device=dev)
flop = 2 * M * 256 * 256
tm = {}
for rnd in range(2):  # alternate, twice: the first timed loop also warms the clock
    for name, fn in (("mfma x@W", lambda: gemm(x, w, 0)), ("torch x@W", lambda: x @ w),
                     ("mfma g@W^T", lambda: gemm(g, w, 1)), ("torch g@W^T", lambda: g @ w.t())):
        tm[name] = t(fn, 20)
res["timing_ms"] = tm
res["TF/s"] = {k: flop / (v * 1e-3) / 1e12 for k, v in tm.items()}
print(json.dumps(res, indent=1))
