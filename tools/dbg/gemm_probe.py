"""x @ W shapes of config 2/3 (M = 2^21, K = N = 256, fp32) under the two
BLAS back ends torch offers on ROCm (hipBLASLt default, rocBLAS)."""
import torch, json
dev = "cuda"
M, K, N = 1 << 21, 256, 256
x = torch.randn(M, K, device=dev)
w = torch.randn(K, N, device=dev) * 0.06
g = torch.randn(M, N, device=dev)


def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def splitk():
    s = M // 8192
    return torch.bmm(x.view(s, 8192, K).transpose(1, 2), g.view(s, 8192, N)).sum(0)


res = {}
for lib in ("hipblaslt", "hipblas", "ck"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        res[lib] = str(e)
        continue
    res[lib] = {"x@W": t(lambda: x @ w), "g@W^T": t(lambda: g @ w.t()), "x^T@g": t(lambda: x.t() @ g),
                "x^T@g splitK": t(splitk)}
flop = 2 * M * K * N
for lib, r in res.items():
    if isinstance(r, dict):
        r.update({k + " TF/s": flop / (v * 1e-3) / 1e12 for k, v in list(r.items())})
print(json.dumps(res, indent=1))
