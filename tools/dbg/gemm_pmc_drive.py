"""Driver for rocprofv3 passes over the MFMA GEMM vs torch.matmul (30 launches each)."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_gemm_probe.so"))
f = lib.mp_gemm_n256_f32
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
              ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
M = 1 << 21
x = torch.randn(M, 256, device="cuda")
w = torch.randn(256, 256, device="cuda") * 0.06
c = torch.empty(M, 256, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(30):
    f(x.data_ptr(), 256, M, 256, w.data_ptr(), 0, 256, c.data_ptr(), 256, s)
for _ in range(30):
    torch.matmul(x, w, out=c)
torch.cuda.synchronize()
print("ok")
