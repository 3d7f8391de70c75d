// Cross-kernel read-after-write probe (r05 root cause of the r04 ln_apply nondeterminism).
//
// One stream, no host synchronisation between launches:
//   for gen in 1..G:  k_write(x, gen)  ;  k_read<MODE>(x, gen, bad[MODE])   (for each MODE in turn)
// k_write stores gen-coded words into a small buffer (rs-sized by default: 2740 rows x 8 B); each
// reader checks every word against the current generation and counts mismatches.  A mismatch is a
// read of data from an EARLIER generation: a cache line that survived the kernel boundaries between
// the writer and the reader.  Readers (all vector loads unless stated):
//   0  plain loads, grid-stride over 514 workgroups (the r04 k_ln_apply_gs geometry)
//   1  plain loads, one workgroup per 8-word row group (the r05 k_ln_apply geometry)
//   2  as 0 with an agent-scope acquire fence (buffer_inv sc1) first
//   3  as 0 with agent-scope relaxed atomic loads (sc1)
//   4  as 0 with a workgroup-scope L1 invalidate (buffer_inv sc0) first
// Usage: coherence [procs=2] [gens=2000] [words=5480] [heavy bytes=0: a streaming copy of that size
// between each write and read] [prime=0: 1 = an LDS-DMA reader of the old values before each write];
// prints one line per process.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <sys/wait.h>
#include <unistd.h>

__device__ __forceinline__ uint32_t code(uint32_t gen, uint32_t i) { return gen * 0x9E3779B1u ^ (i * 2654435761u); }

__global__ void k_write(uint32_t* x, int n, uint32_t gen) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] = code(gen, i);
}

// optional traffic between the writer and the reader (a streaming copy on every CU)
__global__ void k_stream(const uint4* a, uint4* b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// an LDS-DMA reader (as the GEMM engines read their operands): every lane pulls 16 B of x into LDS
// by buffer_load ... lds; the LDS copy is discarded
__global__ void k_prime_lds(const uint32_t* x, int n) {
  __shared__ __attribute__((aligned(16))) uint8_t sm[64 * 16];
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(x), 0, n * 4, 0x00020000);
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int base = (blockIdx.x * 4 + wv) * 256; base < n; base += gridDim.x * 4 * 256)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(sm), 16, (base + lane * 4) * 4, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MODE>
__global__ void k_read(const uint32_t* x, int n, uint32_t gen, unsigned int* bad) {
  if (MODE == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (MODE == 4) asm volatile("buffer_inv sc0" ::: "memory");
  unsigned int miss = 0;
  if (MODE == 1) {
    const int i = blockIdx.x * 8 + (threadIdx.x & 7);
    if (threadIdx.x < 8 && i < n && x[i] != code(gen, i)) miss = 1;
  } else {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      const uint32_t v = MODE == 3 ? __hip_atomic_load(x + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : x[i];
      if (v != code(gen, i)) ++miss;
    }
  }
  if (miss) atomicAdd(bad, miss);
}

static int run(int gens, int n, int64_t heavy, int prime) {
  uint32_t* x = nullptr;
  unsigned int* bad = nullptr;
  uint4 *ha = nullptr, *hb = nullptr;
  if (hipMalloc(&x, n * 4) != hipSuccess || hipMalloc(&bad, 5 * 4) != hipSuccess) return 2;
  if (heavy > 0 && (hipMalloc(&ha, heavy) != hipSuccess || hipMalloc(&hb, heavy) != hipSuccess)) return 2;
  (void)hipMemset(bad, 0, 5 * 4);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int g = 1; g <= gens; ++g) {
    for (int m = 0; m < 5; ++m) {
      if (prime) hipLaunchKernelGGL(k_prime_lds, dim3(514), dim3(256), 0, s, x, n);   // old values, LDS-DMA
      hipLaunchKernelGGL(k_write, dim3(64), dim3(256), 0, s, x, n, (uint32_t)(g * 5 + m));
      if (heavy > 0) hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, s, ha, hb, heavy / 16);
      const uint32_t gen = (uint32_t)(g * 5 + m);
      switch (m) {
        case 0: hipLaunchKernelGGL(k_read<0>, dim3(514), dim3(256), 0, s, x, n, gen, bad + 0); break;
        case 1: hipLaunchKernelGGL(k_read<1>, dim3((n + 7) / 8), dim3(64), 0, s, x, n, gen, bad + 1); break;
        case 2: hipLaunchKernelGGL(k_read<2>, dim3(514), dim3(256), 0, s, x, n, gen, bad + 2); break;
        case 3: hipLaunchKernelGGL(k_read<3>, dim3(514), dim3(256), 0, s, x, n, gen, bad + 3); break;
        case 4: hipLaunchKernelGGL(k_read<4>, dim3(514), dim3(256), 0, s, x, n, gen, bad + 4); break;
      }
    }
  }
  unsigned int h[5] = {0, 0, 0, 0, 0};
  if (hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  printf("pid %d gens %d words %d heavy %lld B prime-by-LDS-DMA %d: stale words read by mode 0 plain/grid-stride %u, 1 plain/row %u, "
         "2 acquire-fence %u, 3 sc1 loads %u, 4 L1-invalidate %u\n",
         (int)getpid(), gens, n, (long long)heavy, prime, h[0], h[1], h[2], h[3], h[4]);
  fflush(stdout);
  (void)hipFree(x);
  (void)hipFree(bad);
  if (ha) (void)hipFree(ha);
  if (hb) (void)hipFree(hb);
  return 0;
}

int main(int argc, char** argv) {
  const int procs = argc > 1 ? atoi(argv[1]) : 2;
  const int gens = argc > 2 ? atoi(argv[2]) : 2000;
  const int n = argc > 3 ? atoi(argv[3]) : 5480;
  const int64_t heavy = argc > 4 ? atoll(argv[4]) : 0;
  const int prime = argc > 5 ? atoi(argv[5]) : 0;
  // fork before any HIP call: each process its own context (as the det_rep processes)
  for (int p = 1; p < procs; ++p)
    if (fork() == 0) return run(gens, n, heavy, prime);
  const int rc = run(gens, n, heavy, prime);
  int st = 0, worst = rc;
  while (wait(&st) > 0)
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) worst = 1;
  return worst;
}
