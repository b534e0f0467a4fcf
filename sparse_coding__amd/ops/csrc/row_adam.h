// Row-wise fused Adam for stacked dictionary parameters (gfx950): the per-row core of the Adam
// kernels (adam.hip).  (A deferred decoder update run by the encoder GEMM after its tiles shared it
// in round 6 -- bit-identical, but slower: scripts/lab/deferred_decoder_adam_r6.patch.)
// Reference semantics: torchopt 0.7.1 `adam` vmapped over the model axis (autoencoders/ensemble.py:
// 94-95, :123, :182-191) with the decoder row normalisation inside the loss (sae_ensemble.py:58-59).
#pragma once
#include "common.h"

namespace scamd {

// Adam bias corrections for 1-based step t, computed on the device so a captured
// HIP graph replays correctly step after step.
__device__ __forceinline__ void bias_corrections(float b1, float b2, int t, float& bc1, float& bc2) {
  bc1 = 1.f - __powf(b1, (float)t);
  bc2 = 1.f - __powf(b2, (float)t);
}

// One dictionary row of the fused Adam, one wave (d = 256 NV): applies the norm Jacobian (norm rows),
// the Adam update, recomputes the row norm and writes the bf16 shadow (normalised for norm rows).
// GBF: the gradient arrives in bf16 (the weight-gradient GEMM's bf16 epilogue): 1/7 of the HBM bytes
// less to read; the moments, the master and the update arithmetic stay fp32.  nsplit > 1: the
// gradient arrives as split-K partial slabs gstride elements apart (summed here).
template <int NV, bool GBF = false>
__device__ __forceinline__ void adam_row_core(float* P, const void* G, float* M, float* V, uint16_t* shadow,
                                              float* norms, long row, int norm, int nsplit, long gstride, float lr,
                                              float b1, float b2, float eps, float bc1, float bc2, int lane) {
  const int d = NV * 256;
  const long base = row * d;
  // NV float4 chunks per lane (d == 256 * NV); compile-time so pv/gv stay in VGPRs.
  const float* P4 = P + base;
  const float* G4 = reinterpret_cast<const float*>(G) + base;
  const uint16_t* GH = reinterpret_cast<const uint16_t*>(G) + base;

  // every load of the row is issued up front (p, g, m, v: 4 NV float4 per lane in flight)
  // so one memory round trip covers the row; the moments do not wait for the norm reductions
  float4 pv[NV], gv[NV], mv_[NV], vv_[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int e = (i * 64 + lane) * 4;
    pv[i] = *reinterpret_cast<const float4*>(P4 + e);
    if constexpr (GBF) {
      const ushort4 h = *reinterpret_cast<const ushort4*>(GH + e);
      gv[i] = make_float4(bf2f(h.x), bf2f(h.y), bf2f(h.z), bf2f(h.w));
    } else {
      gv[i] = *reinterpret_cast<const float4*>(G4 + e);
    }
    mv_[i] = *reinterpret_cast<const float4*>(M + base + e);
    vv_[i] = *reinterpret_cast<const float4*>(V + base + e);
  }
  if (nsplit > 1) {  // split-K partials of the weight-gradient GEMM (few-model shards)
    for (int sp = 1; sp < nsplit; ++sp) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const long e = sp * gstride + (i * 64 + lane) * 4;
        float4 q;
        if constexpr (GBF) {
          const ushort4 h = *reinterpret_cast<const ushort4*>(GH + e);
          q = make_float4(bf2f(h.x), bf2f(h.y), bf2f(h.z), bf2f(h.w));
        } else {
          q = *reinterpret_cast<const float4*>(G4 + e);
        }
        gv[i].x += q.x; gv[i].y += q.y; gv[i].z += q.z; gv[i].w += q.w;
      }
    }
  }
  float ss = 0.f, dot = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    ss += pv[i].x * pv[i].x + pv[i].y * pv[i].y + pv[i].z * pv[i].z + pv[i].w * pv[i].w;
    dot += pv[i].x * gv[i].x + pv[i].y * gv[i].y + pv[i].z * gv[i].z + pv[i].w * gv[i].w;
  }
  float gs = 1.f, ws = 0.f;
  if (norm) {
    ss = wave_sum(ss);
    dot = wave_sum(dot);
    const float nrm = sqrtf(ss);
    if (nrm > 1e-8f) {
      const float inv = 1.f / nrm;
      gs = inv;                 // g' = (g - w_hat <w_hat, g>) / |w|
      ws = dot * inv * inv * inv;  // w_hat <w_hat,g> / |w| = w <w,g> / |w|^3
    } else {
      gs = 1e8f;                // clamp(min=1e-8) has zero derivative below the floor
      ws = 0.f;
    }
  }
  const float omb1 = 1.f - b1, omb2 = 1.f - b2;
  const float step = lr / bc1, rbc2 = 1.f / bc2;
  float ss2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int e = (i * 64 + lane) * 4;
    float4 mv = mv_[i];
    float4 vv = vv_[i];
    float* pp = reinterpret_cast<float*>(&pv[i]);
    float* gg = reinterpret_cast<float*>(&gv[i]);
    float* mm = reinterpret_cast<float*>(&mv);
    float* vvv = reinterpret_cast<float*>(&vv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = gg[k] * gs - pp[k] * ws;
      mm[k] = b1 * mm[k] + omb1 * gk;
      vvv[k] = b2 * vvv[k] + omb2 * gk * gk;
      pp[k] -= step * mm[k] / (sqrtf(vvv[k] * rbc2) + eps);
      ss2 += pp[k] * pp[k];
    }
    *reinterpret_cast<float4*>(M + base + e) = mv;
    *reinterpret_cast<float4*>(V + base + e) = vv;
    *reinterpret_cast<float4*>(P + base + e) = pv[i];
  }
  float sc = 1.f;
  if (norm) {
    ss2 = wave_sum(ss2);
    const float nrm = fmaxf(sqrtf(ss2), 1e-8f);
    sc = 1.f / nrm;
    if (norms && lane == 0) norms[row] = nrm;
  }
  if (shadow) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = (i * 64 + lane) * 4;
      ushort4 h;
      h.x = f2bf(pv[i].x * sc);
      h.y = f2bf(pv[i].y * sc);
      h.z = f2bf(pv[i].z * sc);
      h.w = f2bf(pv[i].w * sc);
      *reinterpret_cast<ushort4*>(shadow + base + e) = h;
    }
  }
}

}  // namespace scamd
