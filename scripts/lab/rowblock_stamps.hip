// Per-step timeline of the row-block fused forward (lab build, not product code): which part of
// each pipeline step (own DMAs landing, the workgroup barrier, the MFMA work) takes the time.
// Headline shapes: G = 8, B = 2048, d = 512, n = 2048.  Prints one JSON line per stamped block.
#ifndef NO_STAMPS
#define SC_RB_STAMPS 1
#endif
#include "sae_rowblock.hip"
#include <stdio.h>
#include <string.h>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(512) void empty_lds_kernel(int* out) {
  __shared__ char sm[161856];
  sm[threadIdx.x] = (char)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && sm[5] == 99) out[blockIdx.x] = 1;
}

static void fill_bf16(uint16_t* d, long n, float scale, unsigned seed) {
  std::vector<uint16_t> h(n);
  unsigned s = seed;
  for (long i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    float f = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * scale;
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = (uint16_t)(u >> 16);
  }
  (void)hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
}

int main() {
  const int G = 8, B = 2048, d = 512, n = 2048;
  uint16_t *x, *we, *wd, *c, *r, *dpre;
  float *bias, *l1, *ep, *dp, *cp;
  void* cmask;
  (void)hipMalloc(&x, (long)B * d * 2);
  (void)hipMalloc(&we, (long)G * n * d * 2);
  (void)hipMalloc(&wd, (long)G * n * d * 2);
  (void)hipMalloc(&c, (long)G * B * n * 2);
  (void)hipMalloc(&dpre, (long)G * B * n * 2);
  (void)hipMalloc(&r, (long)G * B * d * 2);
  (void)hipMalloc(&bias, (long)G * n * 4);
  (void)hipMalloc(&l1, G * 4);
  (void)hipMalloc(&ep, (long)G * (B / 64) * 2 * 4);
  (void)hipMalloc(&dp, (long)G * (B / 64) * 4);
  (void)hipMalloc(&cp, (long)G * (B / 32) * n * 4);
  (void)hipMalloc(&cmask, (long)G * B * n / 8);
  fill_bf16(x, (long)B * d, 8.0f, 1);
  fill_bf16(we, (long)G * n * d, 0.1f, 2);
  fill_bf16(wd, (long)G * n * d, 0.1f, 3);
  (void)hipMemset(bias, 0, (long)G * n * 4);
  (void)hipMemset(l1, 0, G * 4);
  long long* st;
  const long nst = 8l * 1024 * 4;
  (void)hipMalloc(&st, nst * 8);
  long long* null_ptr = nullptr;
#ifndef NO_STAMPS
  (void)hipMemcpyToSymbol(HIP_SYMBOL(scamd::sc_rb_stamps), &null_ptr, sizeof(void*));
#endif
  int stagger = 0, Gl = G, nl = n;
  auto launch = [&] {
    return sc_sae_rowblock(x, 0, we, wd, bias, l1, 256.f, c, r, dpre, cmask, ep, dp, cp, nullptr, Gl, B, nl, d, 0);
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  {
    int* o;
    (void)hipMalloc(&o, 4096);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(empty_lds_kernel, dim3(256), dim3(512), 0, 0, o);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(empty_lds_kernel, dim3(256), dim3(512), 0, 0, o);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"empty_lds_kernel_us\": %.2f}\n", ms * 1e3 / 20);
  }
  for (int nsel : {2048, 256})
  for (int gsel : {8, 1})
    for (int mode : {0}) {
      Gl = gsel;
      nl = nsel;
      stagger = mode;
      for (int i = 0; i < 10; ++i) launch();
      (void)hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("{\"G\": %d, \"n\": %d, \"mode\": %d, \"us_per_launch\": %.2f}\n", Gl, nl, stagger, ms * 1e3 / 20);
    }
  stagger = 1;
  Gl = G;
  nl = n;
#ifdef NO_STAMPS
  (void)st; (void)null_ptr;
  return 0;
#else
  const int U = 48 * (n / 256);
  for (int blk : {0, 1, 37, 255}) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(scamd::sc_rb_stamps), &st, sizeof(void*));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(scamd::sc_rb_block), &blk, sizeof(int));
    (void)hipMemset(st, 0, nst * 8);
    launch();
    (void)hipDeviceSynchronize();
    std::vector<long long> h(nst);
    (void)hipMemcpy(h.data(), st, nst * 8, hipMemcpyDeviceToHost);
    // per phase (enc / dec / dc units) and per wave: mean ticks waiting for DMAs, at the barrier,
    // computing; and the whole loop span
    for (int w : {0, 4}) {
      double sum[3][3] = {{0}}, cnt[3] = {0};
      for (int b = 0; b < U; ++b) {
        const long long* s = &h[((long)w * 1024 + b) * 4];
        int ph = b < 32 * (n / 256) ? (((b & 31) < 16) ? 0 : 1) : 2;
        sum[ph][0] += s[1] - s[0];
        sum[ph][1] += s[2] - s[1];
        sum[ph][2] += s[3] - s[2];
        cnt[ph] += 1;
      }
      const long long span = h[((long)w * 1024 + U - 1) * 4 + 3] - h[((long)w * 1024) * 4];
      printf("{\"block\": %d, \"wave\": %d, \"loop_ticks\": %lld, \"steps\": %d", blk, w, span, U);
      const char* nm[3] = {"enc", "dec", "dc"};
      for (int ph = 0; ph < 3; ++ph)
        printf(", \"%s\": {\"n\": %.0f, \"wait\": %.0f, \"barrier\": %.0f, \"compute\": %.0f}", nm[ph], cnt[ph],
               sum[ph][0] / cnt[ph], sum[ph][1] / cnt[ph], sum[ph][2] / cnt[ph]);
      printf("}\n");
    }
    // first 12 steps of wave 0 raw
    printf("{\"block\": %d, \"raw_wave0\": [", blk);
    for (int b = 0; b < 12; ++b) {
      const long long* s = &h[(long)b * 4];
      printf("%s[%lld, %lld, %lld]", b ? ", " : "", s[1] - s[0], s[2] - s[1], s[3] - s[2]);
    }
    printf("]}\n");
  }
  printf("{\"status\": \"%s\"}\n", hipGetErrorString(hipGetLastError()));
  return 0;
#endif
}
