// Micro-benchmark for the round-4 verdict's lever 1b: fold k_lm_reduce into
// the tail of k_lm_pass with deterministic last-arriver trees, instead of a
// separate reduce launch (csrc/hedge_lm.hip k_lm_pass / k_lm_reduce).
//
// The pass is modelled by its structure only: 256 workgroups of 256 threads,
// the first 64 also write a 40 KB fp32 Gram slab (the euro30 net: P = 106,
// 10 blocks of 32 x 32) and finish `gap` earlier (the real Gram workgroups
// take fewer path blocks), every workgroup writes a 112-float gradient row.
// Path work is a timed wait (s_memrealtime), so only the reduction structure
// differs between the variants:
//   A   pass -> k_red (k_lm_reduce's Gram + packet layout: 160 + 28 WGs) -> consume
//   C   pass folds the packet (16 x 16 last-arriver tree) -> k_red (Gram only) -> consume
//   B2  pass folds both; Gram: 16 groups of 4 slabs, then ONE workgroup sums the 16
//       fp64 partials (the same adds in the same order as A: bitwise)
//   B3  pass folds both; Gram 64 -> 16 -> 4 -> 1 (three last-arriver levels, other order)
//   F   pass -> consume (no reduction at all: the floor)
//   E1  F + every workgroup arrives on a 16 x 16 counter tree (agent-scope release /
//       acquire fences, as the folds), no fold work: the cost of the arrivals alone
//   E2  E1 with workgroup-scope fences (NOT a valid protocol - timing only: the
//       agent-scope release is what writes the slabs back past this XCD's L2)
// consume = one workgroup reading the reduced block (the solve's prologue).
// Every variant runs ITERS sequences in one hipGraph; reported: us per sequence.
//
// build: hipcc --offload-arch=gfx950 -O3 -o lm_fold tools/micro/lm_fold.hip
// run:   ./lm_fold [path_us] [gap_us]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int NG = 10 * 1024;  // Gram entries (10 blocks of 32 x 32)
constexpr int GW = 64;         // Gram workgroups
constexpr int NW = 256;        // pass workgroups
constexpr int R = 112;         // gradient row (P + 4 rounded up)
constexpr int RU = 110;        // entries used
constexpr int ITERS = 50;

struct Bufs {
  float* slab_g;      // [GW][NG]
  float* slab_b;      // [NW][R]
  double* part1;      // [16][NG]  Gram level-1 partials
  double* part2;      // [4][NG]   Gram level-2 partials (B3)
  double* ppart;      // [16][R]   packet level-1 partials
  double* red;        // [NG + R]  reduced block
  unsigned* cnt;      // counters: [0,16) Gram l1, 16 Gram l2, [20,24) Gram l2 (B3), 24 Gram l3, [32,48) packet l1, 48 packet l2
  double* out;
  double inv;
};

__device__ __forceinline__ void busy(unsigned ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// thread 0 adds one arrival; true in every thread of the last arriver (which
// resets the counter: nobody else touches it until the next sequence)
template <bool AGENT = true>
__device__ __forceinline__ bool arrive(unsigned* c, unsigned n, int* sflag) {
  if constexpr (AGENT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == n - 1;
    if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sflag = last;
  }
  __syncthreads();
  const bool last = *sflag != 0;
  if (last) {
    if constexpr (AGENT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  return last;
}

__device__ void fold_packet(const Bufs& b, int w, int* sflag) {
  const int tid = threadIdx.x, grp = w >> 4;
  if (!arrive(b.cnt + 32 + grp, 16, sflag)) return;
  if (tid < R) {
    double a[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) a[u] = (double)b.slab_b[(size_t)(16 * grp + u) * R + tid];
#pragma unroll
    for (int st = 1; st < 16; st <<= 1)
#pragma unroll
      for (int u = 0; u < 16; u += 2 * st) a[u] += a[u + st];
    b.ppart[grp * R + tid] = a[0];
  }
  if (!arrive(b.cnt + 48, 16, sflag)) return;
  if (tid < R) {
    double a[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) a[u] = b.ppart[u * R + tid];
#pragma unroll
    for (int st = 1; st < 16; st <<= 1)
#pragma unroll
      for (int u = 0; u < 16; u += 2 * st) a[u] += a[u + st];
    if (tid < RU) b.red[NG + tid] = a[0];
  }
}

template <bool THREE>
__device__ void fold_gram(const Bufs& b, int w, int* sflag) {
  const int tid = threadIdx.x, g = w & 15;
  if (!arrive(b.cnt + g, 4, sflag)) return;
  // level 1: slabs g, g + 16, g + 32, g + 48 as ((0 + x_g) + x_g+32) + ((0 + x_g+16) + x_g+48)
  const float4* x0 = reinterpret_cast<const float4*>(b.slab_g + (size_t)g * NG);
  const float4* x1 = reinterpret_cast<const float4*>(b.slab_g + (size_t)(g + 16) * NG);
  const float4* x2 = reinterpret_cast<const float4*>(b.slab_g + (size_t)(g + 32) * NG);
  const float4* x3 = reinterpret_cast<const float4*>(b.slab_g + (size_t)(g + 48) * NG);
  double2* p1 = reinterpret_cast<double2*>(b.part1 + (size_t)g * NG);
#pragma unroll 5
  for (int v = tid; v < NG / 4; v += 256) {
    const float4 a = x0[v], c = x1[v], e = x2[v], f = x3[v];
    const double s0x = (0.0 + (double)a.x) + (double)e.x, s1x = (0.0 + (double)c.x) + (double)f.x;
    const double s0y = (0.0 + (double)a.y) + (double)e.y, s1y = (0.0 + (double)c.y) + (double)f.y;
    const double s0z = (0.0 + (double)a.z) + (double)e.z, s1z = (0.0 + (double)c.z) + (double)f.z;
    const double s0w = (0.0 + (double)a.w) + (double)e.w, s1w = (0.0 + (double)c.w) + (double)f.w;
    p1[2 * v] = make_double2(s0x + s1x, s0y + s1y);
    p1[2 * v + 1] = make_double2(s0z + s1z, s0w + s1w);
  }
  if constexpr (!THREE) {
    if (!arrive(b.cnt + 16, 16, sflag)) return;
    // level 2: a = even groups, b = odd groups in order, (a + b) * inv
    const double2* pp = reinterpret_cast<const double2*>(b.part1);
    double2* rd = reinterpret_cast<double2*>(b.red);
    for (int v = tid; v < NG / 2; v += 256) {
      double2 q[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) q[u] = pp[(size_t)u * (NG / 2) + v];
      double ax = 0.0, bx = 0.0, ay = 0.0, by = 0.0;
#pragma unroll
      for (int u = 0; u < 16; u += 2) {
        ax += q[u].x;
        bx += q[u + 1].x;
        ay += q[u].y;
        by += q[u + 1].y;
      }
      rd[v] = make_double2((ax + bx) * b.inv, (ay + by) * b.inv);
    }
  } else {
    const int h = g & 3;
    if (!arrive(b.cnt + 20 + h, 4, sflag)) return;
    const double2* pp = reinterpret_cast<const double2*>(b.part1);
    double2* p2 = reinterpret_cast<double2*>(b.part2 + (size_t)h * NG);
#pragma unroll 4
    for (int v = tid; v < NG / 2; v += 256) {
      const double2 a = pp[(size_t)h * (NG / 2) + v], c = pp[(size_t)(h + 4) * (NG / 2) + v];
      const double2 e = pp[(size_t)(h + 8) * (NG / 2) + v], f = pp[(size_t)(h + 12) * (NG / 2) + v];
      p2[v] = make_double2((a.x + c.x) + (e.x + f.x), (a.y + c.y) + (e.y + f.y));
    }
    if (!arrive(b.cnt + 24, 4, sflag)) return;
    const double2* q2 = reinterpret_cast<const double2*>(b.part2);
    double2* rd = reinterpret_cast<double2*>(b.red);
#pragma unroll 4
    for (int v = tid; v < NG / 2; v += 256) {
      const double2 a = q2[v], c = q2[NG / 2 + v], e = q2[NG + v], f = q2[3 * (NG / 2) + v];
      rd[v] = make_double2(((a.x + c.x) + (e.x + f.x)) * b.inv, ((a.y + c.y) + (e.y + f.y)) * b.inv);
    }
  }
}

// MODE: 0 write only, 1 + packet fold, 2 + Gram fold (two levels), 3 + Gram fold (three levels),
// 4 arrivals only (agent fences), 5 arrivals only (workgroup fences)
template <int MODE>
__global__ __launch_bounds__(256) void k_pass(Bufs b, unsigned t_gram, unsigned t_path, int seq) {
  __shared__ int sflag;
  const int tid = threadIdx.x, w = blockIdx.x;
  const bool gram = w < GW;
  busy(gram ? t_gram : t_path);
  if (tid < R) b.slab_b[(size_t)w * R + tid] = tid < RU ? (float)(((w * 37 + tid * 11 + seq) % 1009) * 1e-3) : 0.f;
  if (gram) {
    float4* s = reinterpret_cast<float4*>(b.slab_g + (size_t)w * NG);
    for (int v = tid; v < NG / 4; v += 256) {
      const int e = 4 * v;
      s[v] = make_float4((float)(((w * 131 + e * 7 + seq) % 997) * 1e-3), (float)(((w * 131 + e * 7 + 7 + seq) % 997) * 1e-3),
                         (float)(((w * 131 + e * 7 + 14 + seq) % 997) * 1e-3), (float)(((w * 131 + e * 7 + 21 + seq) % 997) * 1e-3));
    }
  }
  if constexpr (MODE == 4 || MODE == 5) {
    if (arrive<MODE == 4>(b.cnt + 32 + (w >> 4), 16, &sflag)) arrive<MODE == 4>(b.cnt + 48, 16, &sflag);
    return;
  }
  if constexpr (MODE >= 2)
    if (gram) fold_gram<MODE == 3>(b, w, &sflag);
  if constexpr (MODE >= 1) fold_packet(b, w, &sflag);
}

// k_lm_reduce's layout: Gram WGs (64 entries, 16 x 4 slabs + LDS combine), packet WGs (4 entries, bitrev tree)
template <bool GRAM_ONLY>
__global__ __launch_bounds__(1024) void k_red(Bufs b) {
  __shared__ double part[1024];
  const int tid = threadIdx.x;
  constexpr int NGW = NG / 64;
  if ((int)blockIdx.x < NGW) {
    const int l = tid & 63, g = tid >> 6, e = blockIdx.x * 64 + l;
    const float* col = b.slab_g + e;
    double s0 = 0.0, s1 = 0.0;
    int w = g;
    for (; w + 16 < GW; w += 32) {
      s0 += (double)col[(size_t)w * NG];
      s1 += (double)col[(size_t)(w + 16) * NG];
    }
    if (w < GW) s0 += (double)col[(size_t)w * NG];
    part[tid] = s0 + s1;
    __syncthreads();
    if (g == 0) {
      double a = 0.0, c = 0.0;
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        a += part[q * 64 + l];
        c += part[(q + 1) * 64 + l];
      }
      b.red[e] = (a + c) * b.inv;
    }
    return;
  }
  if (GRAM_ONLY) return;
  const int pw = blockIdx.x - NGW, k = tid & 3, grp = tid >> 2, i = pw * 4 + k;
  const int row = (int)(__builtin_bitreverse32((unsigned)grp) >> 24);
  part[tid] = (double)b.slab_b[(size_t)row * R + i];
  __syncthreads();
#pragma unroll
  for (int st = 128; st >= 1; st >>= 1) {
    if (grp < st) part[tid] += part[tid + 4 * st];
    __syncthreads();
  }
  if (tid < 4 && i < RU) b.red[NG + i] = part[tid];
}

__global__ __launch_bounds__(256) void k_consume(Bufs b) {
  double s = 0.0;
  for (int e = threadIdx.x; e < NG + RU; e += 256) s += b.red[e];
  b.out[threadIdx.x] = s;
}

static double run(const char* name, int variant, Bufs b, unsigned tg, unsigned tp, double* host_red) {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipMemsetAsync(b.cnt, 0, 64 * sizeof(unsigned), st));
  CK(hipMemsetAsync(b.red, 0, (NG + R) * sizeof(double), st));
  CK(hipStreamSynchronize(st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int it = 0; it < ITERS; ++it) {
    switch (variant) {
      case 0:  // A
        hipLaunchKernelGGL(k_pass<0>, dim3(NW), dim3(256), 0, st, b, tg, tp, 0);
        hipLaunchKernelGGL(k_red<false>, dim3(NG / 64 + R / 4), dim3(1024), 0, st, b);
        break;
      case 1:  // C
        hipLaunchKernelGGL(k_pass<1>, dim3(NW), dim3(256), 0, st, b, tg, tp, 0);
        hipLaunchKernelGGL(k_red<true>, dim3(NG / 64), dim3(1024), 0, st, b);
        break;
      case 2:  // B2
        hipLaunchKernelGGL(k_pass<2>, dim3(NW), dim3(256), 0, st, b, tg, tp, 0);
        break;
      case 3:  // B3
        hipLaunchKernelGGL(k_pass<3>, dim3(NW), dim3(256), 0, st, b, tg, tp, 0);
        break;
      case 5:  // E1
        hipLaunchKernelGGL(k_pass<4>, dim3(NW), dim3(256), 0, st, b, tg, tp, 0);
        break;
      case 6:  // E2
        hipLaunchKernelGGL(k_pass<5>, dim3(NW), dim3(256), 0, st, b, tg, tp, 0);
        break;
      default:  // F
        hipLaunchKernelGGL(k_pass<0>, dim3(NW), dim3(256), 0, st, b, tg, tp, 0);
        break;
    }
    hipLaunchKernelGGL(k_consume, dim3(1), dim3(256), 0, st, b);
  }
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 10;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipStreamSynchronize(st));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / (reps * ITERS);
  if (host_red) CK(hipMemcpy(host_red, b.red, (NG + RU) * sizeof(double), hipMemcpyDeviceToHost));
  printf("%-60s %8.2f us per sequence\n", name, us);
  fflush(stdout);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  CK(hipStreamDestroy(st));
  return us;
}

int main(int argc, char** argv) {
  const double path_us = argc > 1 ? atof(argv[1]) : 20.0, gap_us = argc > 2 ? atof(argv[2]) : 3.0;
  const unsigned tp = (unsigned)(path_us * 100.0), tg = (unsigned)((path_us - gap_us) * 100.0);  // 100 MHz ticks
  Bufs b;
  CK(hipMalloc(&b.slab_g, (size_t)GW * NG * 4));
  CK(hipMalloc(&b.slab_b, (size_t)NW * R * 4));
  CK(hipMalloc(&b.part1, (size_t)16 * NG * 8));
  CK(hipMalloc(&b.part2, (size_t)4 * NG * 8));
  CK(hipMalloc(&b.ppart, (size_t)16 * R * 8));
  CK(hipMalloc(&b.red, (size_t)(NG + R) * 8));
  CK(hipMalloc(&b.cnt, 64 * sizeof(unsigned)));
  CK(hipMalloc(&b.out, 256 * 8));
  b.inv = 1.0 / 4096.0;
  printf("pass model: path workgroups %.1f us, Gram workgroups %.1f us earlier; %d sequences per graph\n", path_us,
         gap_us, ITERS);
  static double ra[NG + RU], rx[NG + RU];
  const double f = run("F  pass -> consume (no reduction: floor)", 4, b, tg, tp, nullptr);
  const double a = run("A  pass -> k_red (Gram + packet) -> consume  [current]", 0, b, tg, tp, ra);
  const double c = run("C  pass + packet fold -> k_red (Gram) -> consume", 1, b, tg, tp, rx);
  double dc = 0.0;
  for (int e = 0; e < NG + RU; ++e) dc = fmax(dc, fabs(rx[e] - ra[e]));
  const double b2 = run("B2 pass + packet fold + Gram fold 64->16->1 -> consume", 2, b, tg, tp, rx);
  double d2 = 0.0;
  for (int e = 0; e < NG + RU; ++e) d2 = fmax(d2, fabs(rx[e] - ra[e]));
  const double b3 = run("B3 pass + packet fold + Gram fold 64->16->4->1 -> consume", 3, b, tg, tp, rx);
  double d3 = 0.0;
  for (int e = 0; e < NG + RU; ++e) d3 = fmax(d3, fabs(rx[e] - ra[e]));
  const double e1 = run("E1 pass + arrivals only (agent-scope fences)", 5, b, tg, tp, nullptr);
  const double e2 = run("E2 pass + arrivals only (workgroup fences: timing only)", 6, b, tg, tp, nullptr);
  printf("arrivals over the floor: agent fences %.2f  workgroup fences %.2f us\n", e1 - f, e2 - f);
  printf("reduction cost over the floor: A %.2f  C %.2f  B2 %.2f  B3 %.2f us\n", a - f, c - f, b2 - f, b3 - f);
  printf("max |red - red_A|: C %.3g  B2 %.3g  B3 %.3g (C and B2 add in A's order: 0 expected)\n", dc, d2, d3);
  return 0;
}
