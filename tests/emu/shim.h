// host emulation shim for the lane-walk functions of hpk_decode12.h (one lane at a time)
#pragma once
#include <stdint.h>
#include <algorithm>
#define __device__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static
#define __restrict__
#define HPK_LDS_AS
using std::min; using std::max;
static inline uint32_t __builtin_amdgcn_alignbit(uint32_t a, uint32_t b, uint32_t s) {
    return (uint32_t)((((uint64_t)a << 32) | b) >> (s & 31));
}
static inline uint32_t __builtin_amdgcn_ubfe(uint32_t v, uint32_t off, uint32_t w) {
    off &= 31; w &= 31; if (w == 0) return 0; return (v >> off) & ((1u << w) - 1u) ;
}
static inline uint32_t __builtin_amdgcn_perm(uint32_t a, uint32_t b, uint32_t sel) {
    uint8_t bytes[8]; for (int i=0;i<4;++i){bytes[i]=(b>>(8*i))&255; bytes[4+i]=(a>>(8*i))&255;}
    uint32_t r=0; for(int i=0;i<4;++i){uint32_t s=(sel>>(8*i))&255; uint32_t v = s<8?bytes[s]: (s==12?0:0xFF); r|=v<<(8*i);} return r;
}
static inline uint32_t __clz(uint32_t x){ return x? __builtin_clz(x):32; }
struct uint4 { uint32_t x, y, z, w; };
struct emu_dim3 { uint32_t x = 0, y = 0, z = 0; };
extern emu_dim3 threadIdx, blockIdx;
static inline uint32_t hpk_bswap32(uint32_t x) { return __builtin_bswap32(x); }
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
static inline uint32_t __hip_atomic_fetch_or(uint32_t* p, uint32_t v, int, int) { const uint32_t o = *p; *p = o | v; return o; }
#define HPK_SCHED_FENCE() do { } while (0)
