// EXPERIMENT of round 4 (superseded: the kernel now ships in csrc/mp_gemm.hip as
// mp_gemm_rows_f32, GATConv's row-exact x @ W): a hand-written f32
// MFMA GEMM for the layers' feature transform x @ W (GCNConv /
// GATConv [U5, U6] `torch.matmul(x, self.weight)`) at the configs' shape:
// C[M, 256] = A[M, 256] @ B[256, 256] (B = W or W^T), fp32, on gfx950's f32-input
// MFMA.  Measured (tools/dbg/gemm_mfma_probe.py, M = 2^21): 2.12 ms x@W and
// 2.15 ms g@W^T against hipBLASLt's 2.09 / 2.14 ms -- parity, both at ~84 % of
// the MFMA issue bound at the 2.31 GHz the chip held (GRBM_GUI_ACTIVE / time,
// tools/dbg/gemm_pmc.sh), so torch.matmul stays on the product path.
//
// `v_mfma_f32_32x32x2_f32` runs at the fp32 vector rate (64 FLOP/clk/SIMD, 64
// cycles per instruction) and reads one A and one B value per lane, so operand
// bandwidth is never the limit: the kernel only has to keep the matrix pipe issuing.
//   * B lives in registers: wave w of the 8-wave workgroup owns output columns
//     [32w, 32w + 32) and holds its column block of B for all K as the MFMA B
//     operand (128 VGPRs: lane l, step s -> B[2s + (l >> 5)][32w + (l & 31)]),
//     loaded once per workgroup;
//   * the workgroup is persistent: it walks 64-row tiles of A, each staged in
//     LDS once (double-buffered: the next tile's global loads are in flight
//     while this one is computed) in a k-interleaved image, so a lane's A
//     operands of four consecutive k-steps are one ds_read_b128;
//   * per tile each wave runs 2 row-blocks x 128 k-steps = 256 MFMAs into two
//     independent accumulators; the previous tile's C is stored during the
//     first eight k-groups and the next tile's loads are issued after those
//     stores (vmcnt retires in order).
// Numerics: each output is the k-ordered fmaf chain over k = 0..255 from 0
// (the f32 MFMA's arithmetic): bitwise a sequential fmaf loop (checked).
#include "mp_common.h"

namespace mp {

constexpr int kGemmK = 256;
constexpr int kGemmN = 256;
constexpr int kGemmBM = 64;                     // rows of A per tile
constexpr int kGemmRS = 2 * (kGemmK / 2) + 4;   // LDS row stride (floats) of the k-interleaved image
constexpr int kGemmThreads = 512;               // 8 waves, one per 32-column block

typedef float f32x16 __attribute__((ext_vector_type(16)));

// the k-interleaved image of one A row: k = 2s + h sits at h * 128 + s
__device__ __forceinline__ void gemm_store_lds(float* lds, int row, int k4, const f32x4& v) {
  float* r = lds + row * kGemmRS;
  const int s = k4 * 2;  // k = 4 k4 -> s = 2 k4 (even) and s + 1
  *reinterpret_cast<f32x2*>(r + s) = f32x2{v.x, v.z};          // h = 0: k = 4k4, 4k4 + 2
  *reinterpret_cast<f32x2*>(r + 128 + s) = f32x2{v.y, v.w};    // h = 1: k = 4k4 + 1, 4k4 + 3
}

// BT = false: B is W [256, 256] row-major (C = A W); BT = true: B = W^T, read from
// W row-major (C = A W^T, the input gradient g W^T).  W contiguous.
template <bool BT>
__global__ __launch_bounds__(kGemmThreads, 1) void k_gemm_n256(const float* __restrict__ A, int64_t lda, int64_t M,
                                                              const float* __restrict__ W, float* __restrict__ C,
                                                              int64_t ldc) {
  __shared__ float lds[2][kGemmBM * kGemmRS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int hi = lane >> 5, lo = lane & 31;
  const int64_t n_tiles = (M + kGemmBM - 1) / kGemmBM;

  // B operand of this wave's 32 columns, all 128 k-steps: B[k][n] = W[k][n] or W[n][k]
  float breg[kGemmK / 2];
  {
    const int n = 32 * w + lo;
#pragma unroll
    for (int s = 0; s < kGemmK / 2; ++s) {
      const int k = 2 * s + hi;
      breg[s] = BT ? W[n * kGemmN + k] : W[k * kGemmN + n];
    }
  }
  // retire the B loads here: otherwise the wait-count pass carries them into the
  // tile loop as possibly pending and makes the first MFMAs of every tile wait
  // for the tile prefetch issued just before them (vmcnt counts in order)
  __builtin_amdgcn_s_waitcnt(0);

  // tile loader: 64 rows x 64 float4, 8 per thread in two halves of 4 (each half
  // in flight during one half of the MFMA loop: 16 VGPRs of prefetched data).
  // Wave w loads rows w + 8 j, j = 0..7, lane = float4 column: the row address
  // is wave-uniform (scalar), rows past M are clamped to M - 1 (loaded, never
  // stored), so the loads are unconditional.
  f32x4 pre[4];
  const int ws = __builtin_amdgcn_readfirstlane(w);
  auto load = [&](int64_t tile, int half) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t row = tile * kGemmBM + ws + 8 * (half * 4 + i);
      row = row < M ? row : M - 1;
      pre[i] = *reinterpret_cast<const f32x4*>(A + row * lda + 4 * lane);
    }
  };
  auto stash = [&](float* buf, int half) {
#pragma unroll
    for (int i = 0; i < 4; ++i) gemm_store_lds(buf, w + 8 * (half * 4 + i), lane, pre[i]);
  };

  int64_t tile = blockIdx.x;
  int cur = 0;
  if (tile < n_tiles) {
    load(tile, 0);
    stash(lds[0], 0);
    load(tile, 1);
    stash(lds[0], 1);
  }
  __syncthreads();
  const uint32_t c_off = (uint32_t)(4 * hi * ldc + 32 * w + lo);
  // C of the previous tile, stored during the first eight k-groups of the next
  // one (the stores overlap the MFMAs instead of stalling the whole workgroup)
  f32x16 out0 = {}, out1 = {};
  int64_t out_r0 = -1;
  auto store_part = [&](int part) {  // rows (r & 3) + 8 (r >> 2), r in [2 part, 2 part + 2)
    float* cb = C + out_r0 * ldc;
    if (out_r0 + kGemmBM <= M) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int r = 2 * part + q;
        const int ru = (r & 3) + 8 * (r >> 2);
        cb[(int64_t)ru * ldc + c_off] = out0[r];
        cb[(int64_t)(32 + ru) * ldc + c_off] = out1[r];
      }
    } else {
      const int64_t lim = M - out_r0 - 4 * hi;  // rows ru < lim are in range
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int r = 2 * part + q;
        const int ru = (r & 3) + 8 * (r >> 2);
        if (ru < lim) cb[(int64_t)ru * ldc + c_off] = out0[r];
        if (32 + ru < lim) cb[(int64_t)(32 + ru) * ldc + c_off] = out1[r];
      }
    }
  };
  for (; tile < n_tiles; tile += gridDim.x) {
    const int64_t next = tile + gridDim.x;
    const bool more = next < n_tiles;
    const float* img = lds[cur];
    f32x16 acc0 = {}, acc1 = {};
    const float* a0p = img + lo * kGemmRS + hi * 128;
    const float* a1p = img + (32 + lo) * kGemmRS + hi * 128;
    // A operands one group of four k-steps ahead (the scheduler would otherwise
    // hoist every LDS read of the unrolled loop)
    f32x4 a0n = *reinterpret_cast<const f32x4*>(a0p);
    f32x4 a1n = *reinterpret_cast<const f32x4*>(a1p);
#pragma unroll
    for (int s4 = 0; s4 < kGemmK / 8; ++s4) {
      // k-groups 0..7 store the previous tile's C; the next tile's loads are
      // issued after those stores (vmcnt retires in order: a wait for the loads
      // would otherwise also wait for stores issued after them)
      if (s4 < 8 && out_r0 >= 0) store_part(s4);
      if (s4 == 8 && more) load(next, 0);
      if (s4 == 16 && more) {  // the other buffer takes the first half, the second half loads
        stash(lds[cur ^ 1], 0);
        load(next, 1);
      }
      const f32x4 a0 = a0n, a1 = a1n;
      if (s4 + 1 < kGemmK / 8) {
        a0n = *reinterpret_cast<const f32x4*>(a0p + 4 * (s4 + 1));
        a1n = *reinterpret_cast<const f32x4*>(a1p + 4 * (s4 + 1));
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, breg[4 * s4 + 0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, breg[4 * s4 + 0], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, breg[4 * s4 + 1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, breg[4 * s4 + 1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, breg[4 * s4 + 2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, breg[4 * s4 + 2], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, breg[4 * s4 + 3], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, breg[4 * s4 + 3], acc1, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // C/D map of the 32x32 f32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    out0 = acc0;
    out1 = acc1;
    out_r0 = tile * kGemmBM;
    if (more) stash(lds[cur ^ 1], 1);
    __syncthreads();
    cur ^= 1;
  }
  if (out_r0 >= 0) {
#pragma unroll
    for (int part = 0; part < 8; ++part) store_part(part);
  }
}

}  // namespace mp

using namespace mp;

extern "C" {

int mp_gemm_n256_f32(const float* A, int64_t lda, int64_t M, int32_t K, const float* W, int32_t trans_w,
                     int32_t N, float* C, int64_t ldc, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(K == kGemmK && N == kGemmN, "mp_gemm_n256_f32: only K = N = 256 (got K=%d N=%d)", K, N);
  MP_CHECK_ARG(M >= 0, "mp_gemm_n256_f32: negative M");
  if (M == 0) return MP_OK;
  MP_CHECK_ARG(A && W && C, "mp_gemm_n256_f32: null pointer");
  MP_CHECK_ARG(lda >= K && lda % 4 == 0 && (uintptr_t)A % 16 == 0,
               "mp_gemm_n256_f32: A rows must be 16-byte aligned (lda %% 4 == 0, lda >= K)");
  MP_CHECK_ARG(ldc >= N, "mp_gemm_n256_f32: ldc < N");
  MP_CHECK_ARG(64 * lda < (int64_t)UINT32_MAX && 64 * ldc < (int64_t)UINT32_MAX, "mp_gemm_n256_f32: ld too large");
  int dev = 0, n_cu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t n_tiles = (M + kGemmBM - 1) / kGemmBM;
  const int64_t grid = n_tiles < n_cu ? n_tiles : n_cu;
  if (trans_w)
    k_gemm_n256<true><<<(unsigned)grid, kGemmThreads, 0, as_stream(stream)>>>(A, lda, M, W, C, ldc);
  else
    k_gemm_n256<false><<<(unsigned)grid, kGemmThreads, 0, as_stream(stream)>>>(A, lda, M, W, C, ldc);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
