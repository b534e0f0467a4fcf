// Operand-feed probe (gfx950): how fast can a CU pull bytes that sit in its XCD's L2, in the
// Infinity Cache (MALL) or in HBM, by LDS-DMA (buffer_load_dwordx4 ... lds, the GEMM staging
// path) and by plain global_load_dwordx4 into registers, as a function of bytes in flight?
// Standalone: hipcc --offload-arch=gfx950 -O3 feed_probe.hip -o feed_probe; ./feed_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4_t make_rsrc(const void* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
  r[2] = 0x7FFFFFFF;
  r[3] = 0x00020000;
  return r;
}

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// Each wave streams 1 KiB pieces of its XCD's buffer (blockIdx % 8 -> buffer) into a private
// DEPTH-slot LDS ring, keeping DEPTH-1 pieces in flight.
template <int DEPTH>
__global__ void dma_probe(const char* buf, long buf_bytes, long iters, long* sink) {
  extern __shared__ char smem[];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  const char* base = buf + (long)(blockIdx.x & 7) * buf_bytes;
  const i32x4_t rs = make_rsrc(base);
  const uint32_t voff = lane * 16;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(smem) + wid * DEPTH * 1024);
  const long np = buf_bytes >> 10;
  long p = __builtin_amdgcn_readfirstlane(((blockIdx.x >> 3) * nw + wid) * 37 % np);
  for (long it = 0; it < iters; ++it) {
    const uint32_t soff = (uint32_t)(p << 10);
    const uint32_t dst = lbase + (uint32_t)(it % DEPTH) * 1024;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(dst), "v"(voff), "s"(rs), "s"(soff) : "memory", "m0");
    wait_vm<DEPTH - 1>();
    p += 64 * 8 + 1;
    if (p >= np) p -= np;
  }
  wait_vm<0>();
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = smem[0];
}

// Same stream into registers: DEPTH dwordx4 loads per lane issued back to back, then consumed.
template <int DEPTH>
__global__ void reg_probe(const char* buf, long buf_bytes, long iters, long* sink) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  const char* base = buf + (long)(blockIdx.x & 7) * buf_bytes;
  const long np = buf_bytes >> 10;
  long p = ((blockIdx.x >> 3) * nw + wid) * 37 % np;
  u32x4 acc = {0, 0, 0, 0};
  for (long it = 0; it < iters; it += DEPTH) {
    u32x4 v[DEPTH];
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      v[k] = *reinterpret_cast<const u32x4*>(base + (p << 10) + lane * 16);
      p += 64 * 8 + 1;
      if (p >= np) p -= np;
    }
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) acc ^= v[k];
  }
  if (acc[0] == 0x12345678u && sink) sink[blockIdx.x] = acc[1];
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const long big = 8l * 256 * 1024 * 1024;
  char* buf;
  long* sink;
  hipMalloc(&buf, big);
  hipMalloc(&sink, 1 << 20);
  hipMemset(buf, 1, big);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct Where { const char* name; long bytes; } wheres[] = {{"l2_2MB", 2l << 20}, {"mall_16MB", 16l << 20}, {"hbm_256MB", 256l << 20}};
  for (auto w : wheres) {
    for (int mode = 0; mode < 2; ++mode) {
      for (int nw : {4, 8}) {
        for (int wgpc : {1, 2}) {
          for (int depth : {2, 4, 8, 16}) {
            const int grid = ncu * wgpc;
            // LDS sized so exactly wgpc workgroups fit per CU (160 KiB each)
            const int lds = mode == 0 ? (wgpc == 1 ? 96 * 1024 : 72 * 1024) : (wgpc == 1 ? 96 * 1024 : 72 * 1024);
            if (mode == 0 && nw * depth * 1024 > lds) continue;
            const long iters = 4096;
            auto launch = [&]() {
              if (mode == 0) {
                switch (depth) {
                  case 2: hipLaunchKernelGGL(dma_probe<2>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                  case 4: hipLaunchKernelGGL(dma_probe<4>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                  case 8: hipLaunchKernelGGL(dma_probe<8>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                  case 16: hipLaunchKernelGGL(dma_probe<16>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                }
              } else {
                switch (depth) {
                  case 2: hipLaunchKernelGGL(reg_probe<2>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                  case 4: hipLaunchKernelGGL(reg_probe<4>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                  case 8: hipLaunchKernelGGL(reg_probe<8>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                  case 16: hipLaunchKernelGGL(reg_probe<16>, grid, nw * 64, lds, 0, buf, w.bytes, iters, sink); break;
                }
              }
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            const int reps = 5;
            for (int r = 0; r < reps; ++r) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (double)grid * nw * iters * 1024.0 * reps;
            const double tbs = bytes / (ms * 1e-3) / 1e12;
            printf("{\"where\": \"%s\", \"path\": \"%s\", \"waves\": %d, \"wg_per_cu\": %d, \"depth\": %d, "
                   "\"inflight_kb_per_cu\": %d, \"TBps\": %.2f, \"GBps_per_cu\": %.1f}\n",
                   w.name, mode == 0 ? "ldsdma" : "reg", nw, wgpc, depth, nw * wgpc * (mode == 0 ? depth - 1 : depth),
                   tbs, tbs * 1e3 / ncu);
            fflush(stdout);
          }
        }
      }
    }
  }
  hipError_t e = hipGetLastError();
  printf("{\"status\": \"%s\"}\n", hipGetErrorString(e));
  return 0;
}
