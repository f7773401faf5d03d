// Memory-bound fused elementwise kernels (B2 RMSNorm, B8 SwiGLU, B3+B5 RoPE/KV write).
// All loads/stores are 16-byte vectors (8 bf16); math in fp32.
#include <algorithm>

#include "common.h"

namespace k8s {

// ------------------------------------------------------------ RMSNorm (+add)
// y = rmsnorm(x [+ res]) * w ; when res != nullptr, res <- x + res (bf16).
// One workgroup per row; each thread keeps NC 8-element chunks in registers.
//
// PART: x is the still-unreduced output of a split-K projection GEMM
// (fp32 partials part[s][row][:], s < splits; gemm_mid / grouped layout):
// the row is summed here in the reduce kernels' order and rounded to bf16
// before the residual add, so the result is bit-identical to reduce kernel +
// rmsnorm kernel, one launch (and one [T][H] round trip) fewer.  Every
// decode-step launch costs ~5 us however small (tools/trace_by_grid.py), so
// the launch, not the bytes, is what this saves.
template <int NC, bool PART = false>
__global__ void __launch_bounds__(256) rmsnorm_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ res,
                                                      const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                      int H, int x_stride, int y_stride, float eps,
                                                      const float* __restrict__ part = nullptr, int splits = 0,
                                                      int T = 0) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nv = H >> 3;
  const uint16_t* xr = x + (size_t)row * x_stride;
  uint16_t* rr = res ? res + (size_t)row * H : nullptr;
  // the weight row does not depend on the reduction: issue its loads first
  u16x8 wv[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = threadIdx.x + c * 256;
    if (i < nv) wv[c] = *reinterpret_cast<const u16x8*>(w + i * 8);
  }
  float v[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = threadIdx.x + c * 256;
    if (i < nv) {
      u16x8 a;
      if constexpr (PART) {
        f32x4 a0, a1;
        sum_splits8(part + (size_t)row * H + i * 8, (size_t)T * H, splits, a0, a1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = f2bf(a0[j]);
          a[j + 4] = f2bf(a1[j]);
        }
      } else {
        a = *reinterpret_cast<const u16x8*>(xr + i * 8);
      }
      if (rr) {
        u16x8 b = *reinterpret_cast<const u16x8*>(rr + i * 8);
        u16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float t = bf2f(a[j]) + bf2f(b[j]);
          s[j] = f2bf(t);
          v[c][j] = bf2f(s[j]);
        }
        *reinterpret_cast<u16x8*>(rr + i * 8) = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  const float tot = block_sum(ss, scratch);
  const float inv = rsqrtf(tot / (float)H + eps);
  uint16_t* yr = y + (size_t)row * y_stride;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = threadIdx.x + c * 256;
    if (i < nv) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[c][j] * inv * bf2f(wv[c][j]));
      *reinterpret_cast<u16x8*>(yr + i * 8) = o;
    }
  }
}

// -------------------------------------------------------------- SiLU * up
// gu: [T][2I] (gate | up)  ->  out: [T][I]
__global__ void __launch_bounds__(256) silu_mul_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out,
                                                       int T, int I) {
  const int nv = I >> 3;
  const size_t total = (size_t)T * nv;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const size_t t = idx / nv, i = idx % nv;
    u16x8 g = *reinterpret_cast<const u16x8*>(gu + t * 2 * I + i * 8);
    u16x8 u = *reinterpret_cast<const u16x8*>(gu + t * 2 * I + I + i * 8);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gv = bf2f(g[j]);
      o[j] = f2bf(gv / (1.f + __expf(-gv)) * bf2f(u[j]));
    }
    *reinterpret_cast<u16x8*>(out + t * I + i * 8) = o;
  }
}

// ------------------------------------------------------ RoPE + paged KV write
// qkv: [T][ld] with q heads, then k heads, then v heads (128 dims each).
// Rotates q and k in place (rotate-half / NeoX pairing i <-> i+64), writes
// k -> K page [blk][h][off][:], v -> transposed V page [blk][h][:][off].
// cos_sin: [max_pos][128] fp32 = cos[0..63] | sin[0..63].
//
// PART: the qkv projection was a split-K GEMM whose fp32 partials
// part[s][t][0..ld) (gemm_stream / gemm_mid / grouped layout, s < splits) are
// still unreduced.  Each 8-column piece is summed here in the reduce kernel's
// order (split 0, then += 1, 2, ...) and rounded to bf16 before the rotation,
// and the reduced (then rotated) row is stored back into qkv, so qkv, the K
// page and the V page are bit-identical to reduce kernel + this kernel -- one
// launch and one [T][ld] bf16 round trip fewer per layer of a decode step
// (SURVEY B3 "fuse into the QKV-GEMM epilogue").
template <bool PART>
__device__ __forceinline__ u16x8 qkv_piece(const uint16_t* row, const float* prow, int col, int splits, size_t MN) {
  if constexpr (!PART) {
    return *reinterpret_cast<const u16x8*>(row + col);
  } else {
    f32x4 a0, a1;
    sum_splits8(prow + col, MN, splits, a0, a1);
    u16x8 o;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      o[v] = f2bf(a0[v]);
      o[v + 4] = f2bf(a1[v]);
    }
    return o;
  }
}

// Grid (T, units / block), ONE unit per lane: unit u <
// (nq + nkv) * 8 rotates 8 (i, i + 64) pairs of head u / 8; the next nkv * 16
// units move 8 dims of one v head.  (A block per token looping over its 448
// units left a decode step with ~125 blocks: 9.4 us of serial latency per
// layer at M = 125; spread over ~900 one-wave blocks each lane pays one round
// trip.  Long prefill steps use 256-lane blocks: 64-lane ones measured 7 %
// slower there, dispatch-bound at T x 7 blocks.)
template <bool PART>
__global__ void __launch_bounds__(256) rope_kv_kernel(uint16_t* __restrict__ qkv, int ld, const int* __restrict__ pos,
                                                     const float* __restrict__ cos_sin,
                                                     const int* __restrict__ slots, uint16_t* __restrict__ kc,
                                                     uint16_t* __restrict__ vc, int nq, int nkv, int BS,
                                                     const float* __restrict__ part, int splits, int T) {
  const int t = blockIdx.x;
  const int u = blockIdx.y * blockDim.x + threadIdx.x;
  const int nrot = (nq + nkv) * 8;  // 8 lanes per head, 8 pairs each
  if (u >= nrot + nkv * 16) return;
  uint16_t* row = qkv + (size_t)t * ld;
  const size_t MN = (size_t)T * ld;
  const float* prow = PART ? part + (size_t)t * ld : nullptr;
  const int slot = slots ? slots[t] : -1;
  const int blk = slot >= 0 ? slot / BS : 0, off = slot >= 0 ? slot % BS : 0;
  if (u < nrot) {
    const int hd = u >> 3, c = (u & 7) * 8;
    const float* cs = cos_sin + (size_t)pos[t] * 128;
    uint16_t* xp = row + hd * 128;
    const u16x8 lo = qkv_piece<PART>(row, prow, hd * 128 + c, splits, MN);
    const u16x8 hi = qkv_piece<PART>(row, prow, hd * 128 + 64 + c, splits, MN);
    u16x8 olo, ohi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float co = cs[c + j], si = cs[64 + c + j];
      const float a = bf2f(lo[j]), b = bf2f(hi[j]);
      float ra, rb;
      rope_pair(a, b, co, si, ra, rb);
      olo[j] = f2bf(ra);
      ohi[j] = f2bf(rb);
    }
    *reinterpret_cast<u16x8*>(xp + c) = olo;
    *reinterpret_cast<u16x8*>(xp + 64 + c) = ohi;
    if (hd >= nq && slot >= 0) {
      const int kh = hd - nq;
      uint16_t* kp = kc + (((size_t)blk * nkv + kh) * BS + off) * 128;
      *reinterpret_cast<u16x8*>(kp + c) = olo;
      *reinterpret_cast<u16x8*>(kp + 64 + c) = ohi;
    }
    return;
  }
  // V: 8 dims of one head, transposed scatter into the page (PART: reduced and
  // stored back into qkv first, as the reduce kernel would have)
  if (!PART && slot < 0) return;
  const int i = u - nrot, kh = i >> 4, d0 = (i & 15) * 8;
  const int col = (nq + nkv) * 128 + kh * 128 + d0;
  const u16x8 v = qkv_piece<PART>(row, prow, col, splits, MN);
  if (PART) *reinterpret_cast<u16x8*>(row + col) = v;
  if (slot < 0) return;
  uint16_t* vp = vc + ((size_t)blk * nkv + kh) * 128 * BS + off;
#pragma unroll
  for (int j = 0; j < 8; ++j) vp[(size_t)(d0 + j) * BS] = v[j];
}

}  // namespace k8s

using namespace k8s;

// ------------------------------------------------ graph-step input unpack
// One launch instead of seven D2D copies (each a runtime blit kernel, ~4.5 us
// and ~10 us of host time) before every HIP-graph decode step: the step's flat
// int32 upload [ids | pos | slots | ctx | block table (Bb x mb) | n_items, part |
// items (n_items x 4)] is scattered into the graph's static input buffers.
// spec_src / tok (overlapped steps): row i < n_spec whose spec_src[i] >= 0 takes
// its input id from the device tokens the previous step just sampled,
// max(tok[spec_src[i]], 0) -- the _apply_spec of engine.py in the same launch.
__global__ void __launch_bounds__(256) unpack_step_kernel(const int* __restrict__ flat, int Bb, int mb, int n_items,
                                                          int* __restrict__ ids, int* __restrict__ pos,
                                                          int* __restrict__ slots, int* __restrict__ ctx,
                                                          int* __restrict__ bt, int* __restrict__ n_items_buf,
                                                          int* __restrict__ items, const int* __restrict__ spec_src,
                                                          const int* __restrict__ tok, int n_spec) {
  const int head = 4 * Bb + Bb * mb, total = head + 2 + 4 * n_items;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int v = flat[i];
    if (i < Bb) ids[i] = (i < n_spec && spec_src[i] >= 0) ? max(tok[spec_src[i]], 0) : v;
    else if (i < 2 * Bb) pos[i - Bb] = v;
    else if (i < 3 * Bb) slots[i - 2 * Bb] = v;
    else if (i < 4 * Bb) ctx[i - 3 * Bb] = v;
    else if (i < head) bt[i - 4 * Bb] = v;
    else if (i < head + 2) n_items_buf[i - head] = v;
    else items[i - head - 2] = v;
  }
}

K8S_API int k8s_unpack_step(const void* flat, int Bb, int mb, int n_items, void* ids, void* pos, void* slots,
                            void* ctx, void* bt, void* n_items_buf, void* items, const void* spec_src,
                            const void* tok, int n_spec, hipStream_t s) {
  if (Bb <= 0 || mb <= 0 || n_items < 0 || n_spec < 0 || n_spec > Bb || (n_spec && (!spec_src || !tok)))
    return (int)hipErrorInvalidValue;
  const int total = 4 * Bb + Bb * mb + 2 + 4 * n_items;
  const int grid = std::min((total + 255) / 256, 256);
  hipLaunchKernelGGL(unpack_step_kernel, dim3(grid), dim3(256), 0, s, (const int*)flat, Bb, mb, n_items, (int*)ids,
                     (int*)pos, (int*)slots, (int*)ctx, (int*)bt, (int*)n_items_buf, (int*)items,
                     (const int*)spec_src, (const int*)tok, n_spec);
  return (int)hipGetLastError();
}

K8S_API int k8s_rmsnorm(const void* x, void* res, const void* w, void* y, int T, int H, int x_stride, int y_stride,
                        float eps, hipStream_t s) {
  if (H % 8) return (int)hipErrorInvalidValue;
  const int nc = (H / 8 + 255) / 256;
  const uint16_t* xx = (const uint16_t*)x;
  uint16_t* rr = (uint16_t*)res;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  if (T <= 0) return 0;
  switch (nc) {
    case 1: hipLaunchKernelGGL((rmsnorm_kernel<1, false>), dim3(T), dim3(256), 0, s, xx, rr, ww, yy, H, x_stride, y_stride, eps, nullptr, 0, 0); break;
    case 2: hipLaunchKernelGGL((rmsnorm_kernel<2, false>), dim3(T), dim3(256), 0, s, xx, rr, ww, yy, H, x_stride, y_stride, eps, nullptr, 0, 0); break;
    case 3:
    case 4: hipLaunchKernelGGL((rmsnorm_kernel<4, false>), dim3(T), dim3(256), 0, s, xx, rr, ww, yy, H, x_stride, y_stride, eps, nullptr, 0, 0); break;
    default:
      if (nc > 8) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((rmsnorm_kernel<8, false>), dim3(T), dim3(256), 0, s, xx, rr, ww, yy, H, x_stride, y_stride, eps, nullptr, 0, 0);
  }
  return (int)hipGetLastError();
}

// y = rmsnorm(bf16(sum_s part[s]) + res) * w, res <- bf16(sum_s part[s]) + res;
// part = [splits][T][H] fp32 partials of a split-K GEMM (see rmsnorm_kernel).
K8S_API int k8s_splitk_addnorm(const void* part, int splits, void* res, const void* w, void* y, int T, int H,
                               int y_stride, float eps, hipStream_t s) {
  if (H % 8 || splits < 1 || !part || !res || H / 8 > 1024) return (int)hipErrorInvalidValue;
  if (T <= 0) return 0;
  const int nc = (H / 8 + 255) / 256;
  const float* pp = (const float*)part;
  uint16_t* rr = (uint16_t*)res;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  const uint16_t* nx = nullptr;
  if (nc == 1)
    hipLaunchKernelGGL((rmsnorm_kernel<1, true>), dim3(T), dim3(256), 0, s, nx, rr, ww, yy, H, H, y_stride, eps, pp,
                       splits, T);
  else if (nc == 2)
    hipLaunchKernelGGL((rmsnorm_kernel<2, true>), dim3(T), dim3(256), 0, s, nx, rr, ww, yy, H, H, y_stride, eps, pp,
                       splits, T);
  else
    hipLaunchKernelGGL((rmsnorm_kernel<4, true>), dim3(T), dim3(256), 0, s, nx, rr, ww, yy, H, H, y_stride, eps, pp,
                       splits, T);
  return (int)hipGetLastError();
}

K8S_API int k8s_silu_mul(const void* gu, void* out, int T, int I, hipStream_t s) {
  if (I % 8) return (int)hipErrorInvalidValue;
  if (T <= 0) return 0;
  const size_t total = (size_t)T * (I / 8);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(silu_mul_kernel, dim3(grid), dim3(256), 0, s, (const uint16_t*)gu, (uint16_t*)out, T, I);
  return (int)hipGetLastError();
}

static int rope_block(int T) { return T >= 512 ? 256 : 64; }

K8S_API int k8s_rope_kv(void* qkv, int ld, const int* pos, const float* cos_sin, const int* slots, void* kc, void* vc,
                        int T, int nq, int nkv, int BS, hipStream_t s) {
  if (T <= 0) return 0;
  const int bs = rope_block(T), units = (nq + nkv) * 8 + nkv * 16;
  hipLaunchKernelGGL(rope_kv_kernel<false>, dim3(T, (units + bs - 1) / bs), dim3(bs), 0, s, (uint16_t*)qkv, ld, pos, cos_sin, slots,
                     (uint16_t*)kc, (uint16_t*)vc, nq, nkv, BS, (const float*)nullptr, 0, T);
  return (int)hipGetLastError();
}

// qkv = bf16(sum_s part[s]) with q, k rotated and k, v written to their pages:
// reduce kernel + k8s_rope_kv in one launch, bit-identical.  part =
// [splits][T][ld] fp32 (the split-K GEMM's partials, ld = (nq + 2 nkv) * 128).
K8S_API int k8s_splitk_rope_kv(const void* part, int splits, void* qkv, int ld, const int* pos, const float* cos_sin,
                               const int* slots, void* kc, void* vc, int T, int nq, int nkv, int BS, hipStream_t s) {
  if (T <= 0) return 0;
  if (!part || splits < 1 || ld % 8 || ld < (nq + 2 * nkv) * 128) return (int)hipErrorInvalidValue;
  const int bs = rope_block(T), units = (nq + nkv) * 8 + nkv * 16;
  hipLaunchKernelGGL(rope_kv_kernel<true>, dim3(T, (units + bs - 1) / bs), dim3(bs), 0, s, (uint16_t*)qkv, ld, pos, cos_sin, slots,
                     (uint16_t*)kc, (uint16_t*)vc, nq, nkv, BS, (const float*)part, splits, T);
  return (int)hipGetLastError();
}

// Timed-window marker (bench/rca_bench.py): a one-wave kernel launched at the
// start (tag 1) and end (tag 2) of the benchmark's timed window, so a rocprofv3
// kernel trace can be cut to exactly that window (tools/window_summary.py finds
// it by name and grid).  It writes nothing.
__global__ void window_mark_kernel(int tag) {
  if (tag < 0) asm volatile("s_nop 0");
}

K8S_API int k8s_window_mark(int tag, hipStream_t s) {
  hipLaunchKernelGGL(window_mark_kernel, dim3(tag), dim3(64), 0, s, tag);
  return (int)hipGetLastError();
}

// Debug (knob nonfinite_check): flag[0] = 1 when any of the n bf16 values is
// NaN or inf (exponent all ones).  The engine passes one flag per layer and
// reads them with the step's sampled tokens: no host sync of its own.  Every
// offending lane stores the same 1 (plain vector store).
__global__ void __launch_bounds__(256) nonfinite_flag_kernel(const uint16_t* __restrict__ x, long n,
                                                             int* __restrict__ flag) {
  const long n8 = n / 8;
  bool bad = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + i * 8);
#pragma unroll
    for (int c = 0; c < 8; ++c) bad |= (v[c] & 0x7F80u) == 0x7F80u;
  }
  if (blockIdx.x == 0 && threadIdx.x < n - n8 * 8) bad |= (x[n8 * 8 + threadIdx.x] & 0x7F80u) == 0x7F80u;
  if (bad) flag[0] = 1;
}

K8S_API int k8s_nonfinite_flag(const void* x, long n, int* flag, hipStream_t s) {
  if (n <= 0) return 0;
  if (!x || !flag || ((uintptr_t)x % 16)) return (int)hipErrorInvalidValue;
  const long blocks = std::min<long>(512, (n / 8 + 255) / 256 + 1);
  hipLaunchKernelGGL(nonfinite_flag_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint16_t*)x, n, flag);
  return (int)hipGetLastError();
}

// Host-visible completion flag (knob token_flag): stream-ordered after the
// sampled tokens' device -> host copy, every lane of one wave stores `value`
// into its own int of `flag` (pinned host memory; plain per-lane VECTOR
// stores, no scalar-cache write), and the engine polls flag[0] with short
// sleeps instead of waiting in hipEventSynchronize (engine/sampler.py).  The
// copy has completed before this kernel starts (stream order), so a host that
// reads flag[0] >= value also reads the step's tokens.
__global__ void __launch_bounds__(64) host_flag_kernel(int* __restrict__ flag, int value) {
  // a system-scope release store per lane: write-through to host memory (sc0 sc1)
  __hip_atomic_store(flag + threadIdx.x, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

K8S_API int k8s_host_flag(int* flag, int value, hipStream_t s) {
  if (!flag) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(host_flag_kernel, dim3(1), dim3(64), 0, s, flag, value);
  return (int)hipGetLastError();
}
