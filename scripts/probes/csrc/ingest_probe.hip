// Per-CU ingest probe: every workgroup (one per CU, 8 waves) streams its own
// slice of an L2/MALL-resident buffer `reps` times, either by LDS-DMA
// (buffer_load_dwordx4 ... lds into a 4-stage ring, counted vmcnt) or by
// buffer_load_dwordx4 into VGPRs (summed so the loads stay live).  Prints
// GB/s per CU and for the chip.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline rsrc_t mk(const void* base, uint32_t bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  void* ub = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// MODE 0: LDS-DMA, 1 KiB per wave-instruction, 8 in flight per wave
// MODE 1: VGPR loads, 16 B per lane, 8 in flight per wave
template <int MODE>
__global__ void __launch_bounds__(512) ingest(const float* buf, uint32_t slice_bytes, int reps,
                                              float* sink) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[8 * 8 * 1024];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const unsigned char* base = reinterpret_cast<const unsigned char*>(buf) + (size_t)blockIdx.x * slice_bytes;
  const rsrc_t r = mk(base, slice_bytes);
  const int per_wave = slice_bytes / 8;  // bytes this wave streams per rep
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int rep = 0; rep < reps; ++rep) {
    for (int off = 0; off < per_wave; off += 8 * 1024) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = wave * per_wave + off + u * 1024 + lane * 16;
        if (MODE == 0) {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(uintptr_t)(lds + (wave * 8 + u) * 1024), 16, o, 0, 0, 0);
        } else {
          acc += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
        }
      }
      if (MODE == 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (MODE == 1 && acc[0] == 12345.f) sink[threadIdx.x] = acc[1] + acc[2] + acc[3];
}

int main() {
  int cus = 256;
  const uint32_t slice = 256 * 1024;  // per CU; 64 MB total (L2 + MALL resident)
  float* buf; float* sink;
  hipMalloc(&buf, (size_t)slice * cus);
  hipMalloc(&sink, 4096);
  hipMemset(buf, 0, (size_t)slice * cus);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int sl : {16 * 1024, 64 * 1024, 256 * 1024}) {
    const int reps = (int)(64ll * 1024 * 1024 / sl);
    for (int mode = 0; mode < 2; ++mode) {
      for (int it = 0; it < 2; ++it) {
        hipEventRecord(a);
        if (mode == 0) hipLaunchKernelGGL(ingest<0>, dim3(cus), dim3(512), 0, 0, buf, (uint32_t)sl, reps, sink);
        else hipLaunchKernelGGL(ingest<1>, dim3(cus), dim3(512), 0, 0, buf, (uint32_t)sl, reps, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        const double bytes = (double)sl * reps;
        if (it) printf("slice %6d KB  %s  %.1f GB/s per CU  %.2f TB/s chip\n", sl / 1024,
                       mode ? "vgpr   " : "lds-dma", bytes / (ms * 1e-3) / 1e9,
                       bytes * cus / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
