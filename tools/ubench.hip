// Latency micro-benchmarks for the serial recode chain (gfx950): cycles per dependent operation
// for one wave, measured with s_memtime.  hipcc --offload-arch=gfx950 -O3 tools/ubench.hip -o /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define N 4096
__device__ __forceinline__ uint64_t clk() {
  uint64_t t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

__global__ void k_salu(uint64_t* out, uint32_t seed) {
  uint32_t x = seed;
  uint64_t t0 = clk();
  for (int i = 0; i < N; i++) {
    asm volatile("s_add_u32 %0, %0, 3\n s_xor_b32 %0, %0, 5\n s_lshl_b32 %0, %0, 1\n s_and_b32 %0, %0, 0xffff"   : "+s"(x) :: "scc");
  }
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = x; }
}
__global__ void k_salu_indep(uint64_t* out, uint32_t seed) {
  uint32_t x = seed, y = seed + 1, z = seed + 2, w = seed + 3;
  uint64_t t0 = clk();
  for (int i = 0; i < N; i++) {
    asm volatile("s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 3\n s_add_u32 %2, %2, 3\n s_add_u32 %3, %3, 3" : "+s"(x), "+s"(y), "+s"(z), "+s"(w) :: "scc");
  }
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = x + y + z + w; }
}
__global__ void k_valu(uint64_t* out, uint32_t seed) {
  uint32_t x = seed + threadIdx.x;
  uint64_t t0 = clk();
  for (int i = 0; i < N; i++) {
    asm volatile("v_add_u32 %0, %0, 3\n v_xor_b32 %0, %0, 5\n v_lshlrev_b32 %0, 1, %0\n v_and_b32 %0, 0xffff, %0" : "+v"(x));
  }
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = x; }
}
__global__ void k_lds(uint64_t* out, uint32_t seed) {
  __shared__ uint32_t t[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) t[i] = (i * 7 + 13) & 1023;
  __syncthreads();
  uint32_t x = seed & 1023;
  uint64_t t0 = clk();
  for (int i = 0; i < N / 4; i++) {
    x = t[x];
    x = __builtin_amdgcn_readfirstlane(x);
  }
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = (t1 - t0) * 4; out[blockIdx.x * 2 + 1] = x; }
}
__global__ void k_readlane(uint64_t* out, uint32_t seed) {
  uint32_t v = (threadIdx.x * 7 + 13) & 63;
  uint32_t x = seed & 63;
  uint64_t t0 = clk();
  for (int i = 0; i < N / 4; i++) x = __builtin_amdgcn_readlane(v, x);
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = (t1 - t0) * 4; out[blockIdx.x * 2 + 1] = x; }
}
__global__ void k_valu_to_salu(uint64_t* out, uint32_t seed) {
  uint32_t x = seed;
  uint64_t t0 = clk();
  for (int i = 0; i < N / 4; i++) {
    uint32_t v;
    asm volatile("v_add_u32 %0, %1, 1" : "=v"(v) : "s"(x));
    x = __builtin_amdgcn_readfirstlane(v);
  }
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = (t1 - t0) * 4; out[blockIdx.x * 2 + 1] = x; }
}
__global__ void k_branch(uint64_t* out, uint32_t seed) {
  uint32_t x = seed;
  uint64_t t0 = clk();
  for (int i = 0; i < N; i++) {
    asm volatile("s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 1f\n s_add_u32 %0, %0, 1\n1:\n" : "+s"(x) :: "scc");
  }
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = x; }
}

// dependent scalar loads from a small constant table (scalar-cache hits): the recoded decoder's
// reciprocal lookup
__global__ void k_sload(uint64_t* out, uint32_t seed, const uint32_t* tab) {
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  cu32* t = (cu32*)tab;
  uint32_t x = seed & 255;
  uint64_t t0 = clk();
  for (int i = 0; i < N / 4; i++) x = t[x] & 255;
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = (t1 - t0) * 4; out[blockIdx.x * 2 + 1] = x; }
}
__global__ void k_branch_taken(uint64_t* out, uint32_t seed) {
  uint32_t x = seed;
  uint64_t t0 = clk();
  for (int i = 0; i < N; i++) {
    asm volatile("s_cmp_lg_u32 %0, 12345\n s_cbranch_scc1 1f\n s_nop 0\n1:\n s_add_u32 %0, %0, 1\n" : "+s"(x) :: "scc");
  }
  uint64_t t1 = clk();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = x; }
}
static uint32_t* g_tab;
static void k_sload_launch(uint64_t* d, uint32_t seed, int blocks) {
  hipLaunchKernelGGL(k_sload, dim3(blocks), dim3(64), 0, 0, d, seed, g_tab);
}

int main() {
  uint64_t* d;
  (void)hipMalloc(&d, 2048 * 16);
  uint64_t h[4096];
  struct K { const char* name; void (*f)(uint64_t*, uint32_t); int per; } ks[] = {
    {"salu dep (4 ops/iter)", k_salu, 4}, {"salu 4 indep chains", k_salu_indep, 4}, {"valu dep (4 ops/iter)", k_valu, 4},
    {"lds dep read + readfirstlane", k_lds, 1}, {"v_readlane dep", k_readlane, 1}, {"valu->readfirstlane->salu", k_valu_to_salu, 1},
    {"s_cmp+s_cbranch(not taken)+s_add", k_branch, 3}, {"s_cmp+s_cbranch(taken)+s_add", k_branch_taken, 3}};
  setvbuf(stdout, nullptr, _IONBF, 0);
  {
    uint32_t ht[256];
    for (int i = 0; i < 256; i++) ht[i] = (uint32_t)((i * 97 + 31) & 255);
    (void)hipMalloc(&g_tab, sizeof(ht));
    (void)hipMemcpy(g_tab, ht, sizeof(ht), hipMemcpyHostToDevice);
    for (int blocks : {1, 1024}) {
      k_sload_launch(d, 1, blocks);
      (void)hipDeviceSynchronize();
      k_sload_launch(d, 1, blocks);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      (void)hipMemcpy(h, d, blocks * 16, hipMemcpyDeviceToHost);
      double s = 0;
      for (int b = 0; b < blocks; b++) s += h[2 * b];
      printf("%-40s waves=%5d  cycles/op = %.2f\n", "s_load dep (scalar cache)", blocks, s / blocks / N);
    }
  }
  for (auto& k : ks) {
    for (int blocks : {1, 256, 1024, 2048}) {
      printf("# %s %d\n", k.name, blocks);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d, 1);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d, 1);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      (void)hipMemcpy(h, d, blocks * 16, hipMemcpyDeviceToHost);
      double s = 0;
      for (int b = 0; b < blocks; b++) s += h[2 * b];
      printf("%-40s waves=%5d  cycles/op = %.2f\n", k.name, blocks, s / blocks / N / k.per * (k.per == 1 ? 1 : 1));
    }
  }
  return 0;
}
