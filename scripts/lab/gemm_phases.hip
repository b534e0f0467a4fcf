// Per-workgroup phase timing of the step GEMMs (gfx950 lab build, not product code):
// SC_PHASE_STAMPS makes sae_gemm_kernel stamp s_memtime at kernel entry, when its first K-tile
// has landed, after the K loop and after the epilogue (into a buffer of its own).  Shapes are
// the headline step's (G = 8, B = 2048, d = 512, n = 2048): encoder (EPI_ENC, 128x128),
// decoder (EPI_DEC, 128x128) and both weight gradients (EPI_F32, 256x256).
#define SC_PHASE_STAMPS 1
#include "../../sparse_coding__amd/ops/csrc/sae_gemm_kernel.h"
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

using namespace scamd;

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

struct Stat { double med, p10, p90; };
static Stat stat(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  auto q = [&](double f) { return v[(size_t)(f * (v.size() - 1))]; };
  return {q(0.5), q(0.1), q(0.9)};
}

static const char* g_raw_dir = nullptr;  // argv[1]: per-block raw stamps as CSV (one file per kernel)

template <class F>
static void run(const char* name, long nblocks, F launch) {
  long long* st;
  (void)hipMalloc(&st, nblocks * 8 * sizeof(long long));
  long long* sub;
  (void)hipMalloc(&sub, nblocks * 8 * sizeof(long long));
  (void)hipMemset(sub, 0, nblocks * 8 * sizeof(long long));
  long long* null_ptr = nullptr;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_sub_buf), &null_ptr, sizeof(void*));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_stamp_buf), &null_ptr, sizeof(void*));
  for (int i = 0; i < 20; ++i) launch();  // warm (clocks, caches)
  (void)hipEventRecord(e0);
  for (int i = 0; i < 20; ++i) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_stamp_buf), &st, sizeof(void*));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_sub_buf), &sub, sizeof(void*));
  launch();
  (void)hipDeviceSynchronize();
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_sub_buf), &null_ptr, sizeof(void*));
  std::vector<long long> h(nblocks * 8), hs(nblocks * 8);
  (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hs.data(), sub, hs.size() * 8, hipMemcpyDeviceToHost);
  // memtime ticks per ns from the whole launch's realtime (100 MHz) span
  long long t0 = h[0], tmax = 0, r0 = h[4], rmax = 0;
  for (long b = 0; b < nblocks; ++b) {
    t0 = std::min(t0, h[b * 8]);
    r0 = std::min(r0, h[b * 8 + 4]);
    tmax = std::max(tmax, h[b * 8 + 3]);
    rmax = std::max(rmax, h[b * 8 + 5]);
  }
  const double ghz = (double)(tmax - t0) / ((double)(rmax - r0) * 10.0);
  std::vector<double> start, fill, kloop, epi, life;
  for (long b = 0; b < nblocks; ++b) {
    const long long* s = &h[b * 8];
    start.push_back((s[0] - t0) / ghz / 1e3);
    fill.push_back((s[1] - s[0]) / ghz / 1e3);
    kloop.push_back((s[2] - s[1]) / ghz / 1e3);
    epi.push_back((s[3] - s[2]) / ghz / 1e3);
    life.push_back((s[3] - s[0]) / ghz / 1e3);
  }
  if (g_raw_dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/%s.csv", g_raw_dir, name);
    FILE* fo = fopen(path, "w");
    if (fo) {
      fprintf(fo, "block,t0,t1,t2,t3,rt0,rt3,hw_id,xcc_id,e0,e1,e2,e3,e4,e5,e6\n");
      for (long b = 0; b < nblocks; ++b) {
        const long long* s = &h[b * 8];
        const long long* e = &hs[b * 8];
        fprintf(fo, "%ld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld\n", b, s[0], s[1], s[2],
                s[3], s[4], s[5], s[6], s[7], e[0], e[1], e[2], e[3], e[4], e[5], e[6]);
      }
      fclose(fo);
    }
  }
  Stat a = stat(start), f = stat(fill), k = stat(kloop), e = stat(epi), l = stat(life);
  printf("{\"kernel\": \"%s\", \"blocks\": %ld, \"us_per_launch\": %.2f, \"stamped_span_us\": %.2f, \"clock_ghz\": %.3f, "
         "\"start_us\": [%.2f, %.2f, %.2f], \"fill_us\": [%.2f, %.2f, %.2f], \"kloop_us\": [%.2f, %.2f, %.2f], "
         "\"epilogue_us\": [%.2f, %.2f, %.2f], \"lifetime_us\": [%.2f, %.2f, %.2f]}\n",
         name, nblocks, ms * 1e3 / 20, (tmax - t0) / ghz / 1e3, ghz, a.p10, a.med, a.p90, f.p10, f.med, f.p90,
         k.p10, k.med, k.p90, e.p10, e.med, e.p90, l.p10, l.med, l.p90);
  fflush(stdout);
  (void)hipFree(st);
  (void)hipFree(sub);
}

int main(int argc, char** argv) {
  if (argc > 1) g_raw_dir = argv[1];
  const int G = 8, B = 2048, d = 512, n = 2048;
  uint16_t *x, *we, *wd, *c, *r;
  float *bias, *part, *g;
  uint64_t* cmask;
  (void)hipMalloc(&x, (long)B * d * 2);
  (void)hipMalloc(&we, (long)G * n * d * 2);
  (void)hipMalloc(&wd, (long)G * n * d * 2);
  (void)hipMalloc(&c, (long)G * B * n * 2);
  (void)hipMalloc(&r, (long)G * B * d * 2);
  (void)hipMalloc(&bias, (long)G * n * 4);
  (void)hipMalloc(&part, (long)G * (B / 128) * (n / 128) * 2 * 4);
  (void)hipMalloc(&g, 2l * G * n * d * 4);
  (void)hipMalloc(&cmask, (long)G * B * n / 8);
  fill_bf16(x, (long)B * d, 8.0f, 1);
  fill_bf16(we, (long)G * n * d, 0.1f, 2);
  fill_bf16(wd, (long)G * n * d, 0.1f, 3);
  fill_bf16(c, (long)G * B * n, 1.0f, 4);
  fill_bf16(r, (long)G * B * d, 1.0f, 5);
  (void)hipMemset(bias, 0, (long)G * n * 4);

  {  // encoder: c = relu(x We^T + b), 128x128
    GemmParams p{};
    p.prob[0].a[0] = p.prob[0].a[1] = {x, d, 0};
    p.prob[0].b[0] = p.prob[0].b[1] = {we, d, (long)n * d};
    p.prob[0].c = c; p.prob[0].alpha = 1.f; p.nprob = 1;
    p.M = B; p.N = n; p.K1 = d; p.K2 = 0; p.G = G; p.ldc = n; p.sc = (long)B * n;
    p.bias = bias; p.sbias = n; p.part = part; p.cmask = cmask; p.ksplit = 1;
#if defined(LAB_256x128)
    run("enc_256x128", n_blocks<S256x128>(B, n, G, 1), [&] { launch<S256x128, 64, 2>(EPI_ENC, true, true, p, 1, 0); });
    run("nt_bf16_256x128", n_blocks<S256x128>(B, n, G, 1), [&] { launch<S256x128, 64, 2>(EPI_BF16, true, true, p, 1, 0); });
    run("enc_128_bk32x3", n_blocks<S128>(B, n, G, 1), [&] { launch<S128, 32, 3, false, true>(EPI_ENC, true, true, p, 1, 0); });
#elif !defined(LAB_BIG)
    // the product's encoder configuration (cfg 29: 128x128, BK32 x 3 ring, software-pipelined loop)
    run("enc_128_p32", n_blocks<S128>(B, n, G, 1), [&] { launch<S128, 32, 3, false, true>(EPI_ENC, true, true, p, 1, 0); });
    run("enc_128_bk32x3", n_blocks<S128>(B, n, G, 1), [&] { launch<S128, 32, 3, false>(EPI_ENC, true, true, p, 1, 0); });
    run("enc_128", n_blocks<S128>(B, n, G, 1), [&] { launch<S128, 64, 2>(EPI_ENC, true, true, p, 1, 0); });
#else
    run("enc_256", n_blocks<S256>(B, n, G, 1), [&] { launch<S256, 64, 2>(EPI_ENC, true, true, p, 1, 0); });
#endif
  }
#ifndef LAB_256x128
  {  // decoder: R = c Wd - x, 128x128
    GemmParams p{};
    p.prob[0].a[0] = p.prob[0].a[1] = {c, n, (long)B * n};
    p.prob[0].b[0] = p.prob[0].b[1] = {wd, d, (long)n * d};
    p.prob[0].c = r; p.prob[0].alpha = 1.f; p.nprob = 1;
    p.M = B; p.N = d; p.K1 = n; p.K2 = 0; p.G = G; p.ldc = d; p.sc = (long)B * d;
    p.aux = x; p.ldaux = d; p.saux = 0; p.part = part; p.ksplit = 1;
#ifndef LAB_BIG
    run("dec_128", n_blocks<S128>(B, d, G, 1), [&] { launch<S128, 64, 2>(EPI_DEC, true, false, p, 1, 0); });
#endif
  }
#ifdef LAB_MASKED
  {  // masked decoder (the masked-ensemble config: live sizes 512 * linspace(1, 5, 8) of a 2560 stack,
     // K range cut per model on the device): which blocks share a CU, and how long each CU is busy
    const int ns = 2560;
    uint16_t *cm, *wm;
    int* nact;
    const int live[8] = {512, 804, 1097, 1389, 1682, 1974, 2267, 2560};
    (void)hipMalloc(&cm, (long)G * B * ns * 2);
    (void)hipMalloc(&wm, (long)G * ns * d * 2);
    (void)hipMalloc(&nact, 8 * 4);
    (void)hipMemcpy(nact, live, sizeof live, hipMemcpyHostToDevice);
    fill_bf16(cm, (long)G * B * ns, 1.0f, 6);
    fill_bf16(wm, (long)G * ns * d, 0.1f, 7);
    GemmParams p{};
    p.prob[0].a[0] = p.prob[0].a[1] = {cm, ns, (long)B * ns};
    p.prob[0].b[0] = p.prob[0].b[1] = {wm, d, (long)ns * d};
    p.prob[0].c = r; p.prob[0].alpha = 1.f; p.nprob = 1;
    p.M = B; p.N = d; p.K1 = ns; p.K2 = 0; p.G = G; p.ldc = d; p.sc = (long)B * d;
    p.aux = x; p.ldaux = d; p.saux = 0; p.part = part; p.ksplit = 1; p.nact_k = nact;
    run("dec_masked", n_blocks<S128>(B, d, G, 1), [&] { launch<S128, 64, 2>(EPI_DEC, true, false, p, 1, 0); });
    p.nact_k = nullptr;
    run("dec_unmasked2560", n_blocks<S128>(B, d, G, 1), [&] { launch<S128, 64, 2>(EPI_DEC, true, false, p, 1, 0); });
  }
#endif
  {  // code gradient: dpre = 1[c > 0] (R Wd^T + l d / 2), activity from the bitmask, 128x128 BK32x3
    GemmParams p{};
    float* l1;
    float* colpart;
    (void)hipMalloc(&l1, G * 4);
    (void)hipMalloc(&colpart, (long)G * (B / 128) * n * 4);
    (void)hipMemset(l1, 0, G * 4);
    p.prob[0].a[0] = p.prob[0].a[1] = {r, d, (long)B * d};
    p.prob[0].b[0] = p.prob[0].b[1] = {wd, d, (long)n * d};
    p.prob[0].c = c; p.prob[0].alpha = 1.f; p.nprob = 1;
    p.M = B; p.N = n; p.K1 = d; p.K2 = 0; p.G = G; p.ldc = n; p.sc = (long)B * n;
    p.colpart = colpart; p.l1 = l1; p.l1_add_scale = d / 2.0f; p.cmask = cmask; p.ksplit = 1;
#ifndef LAB_BIG
    run("dc_128_p32", n_blocks<S128>(B, n, G, 1), [&] { launch<S128, 32, 3, false, true>(EPI_DC_MASK, true, true, p, 1, 0); });
    run("dc_128_bk32x3", n_blocks<S128>(B, n, G, 1), [&] { launch<S128, 32, 3, false>(EPI_DC_MASK, true, true, p, 1, 0); });
#endif
  }
  {  // weight gradients: dWd = c^T R, dWe = c^T x (stand-in for dpre), 256x256, two problems
    GemmParams p{};
    p.prob[0].a[0] = p.prob[0].a[1] = {c, n, (long)B * n};
    p.prob[0].b[0] = p.prob[0].b[1] = {r, d, (long)B * d};
    p.prob[0].c = g; p.prob[0].alpha = 1.f;
    p.prob[1].a[0] = p.prob[1].a[1] = {c, n, (long)B * n};
    p.prob[1].b[0] = p.prob[1].b[1] = {x, d, 0};
    p.prob[1].c = g + (long)G * n * d; p.prob[1].alpha = 1.f;
    p.nprob = 2;
    p.M = n; p.N = d; p.K1 = B; p.K2 = 0; p.G = G; p.ldc = d; p.sc = (long)n * d; p.ksplit = 1;
#ifdef LAB_BIG
    run("wgrad_256", n_blocks<S256>(n, d, G, 2), [&] { launch<S256, 64, 2>(EPI_F32, false, false, p, 2, 0); });
#else
    run("wgrad_128", n_blocks<S128>(n, d, G, 2), [&] { launch<S128, 64, 2>(EPI_F32, false, false, p, 2, 0); });
#endif
  }
#endif
  printf("{\"status\": \"%s\"}\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
