// Basic types and qualifiers shared by the device arithmetic headers.
// The headers compile as HIP device code (hipcc, gfx950) for the product and,
// for host-side debugging tests only, as plain C++ (g++).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BGV_HD __host__ __device__ __forceinline__
#define BGV_HDN __host__ __device__ __noinline__
#define BGV_CONST __constant__ const
#define BGV_NI static __host__ __device__ __noinline__
#ifndef BGV_FP2_INLINE
#define BGV_FP2_INLINE 0
#endif
#if BGV_FP2_INLINE
#define BGV_NI2 BGV_HD
#else
#define BGV_NI2 BGV_NI
#endif
#else
#define BGV_HD static inline
#define BGV_HDN static
#define BGV_CONST static const
#define BGV_NI static inline
#define BGV_NI2 static inline
#endif

namespace bgv {

constexpr int NL = 12;  // 32-bit limbs per Fp element (384 bits)

struct fp_t { uint32_t l[NL]; };
struct fp2_t { fp_t c0, c1; };
struct fp6_t { fp2_t c0, c1, c2; };
struct fp12_t { fp6_t c0, c1; };

// Jacobian points (x = X/Z^2, y = Y/Z^3); Z == 0 is the point at infinity
struct g1j_t { fp_t x, y, z; };
struct g1a_t { fp_t x, y; };
struct g2j_t { fp2_t x, y, z; };
struct g2a_t { fp2_t x, y; };

}  // namespace bgv
