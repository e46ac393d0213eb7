// LDS address-space access for the cooperative kernels (device only).
// Their exchange buffers are __shared__, but the helpers that use them take
// plain pointers; through a generic pointer every access is a flat
// load/store, which waits on both the vector-memory and the LDS counters.
// Casting to the LDS address space gives ds_read / ds_write.
#pragma once
#include "bls_types.h"

#define BGV_LDS __attribute__((address_space(3)))

namespace bgv {

__device__ __forceinline__ fp_t lds_get(const BGV_LDS fp_t* p) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < NL; k++) r.l[k] = p->l[k];
  return r;
}
__device__ __forceinline__ void lds_put(BGV_LDS fp_t* p, const fp_t& v) {
#pragma unroll
  for (int k = 0; k < NL; k++) p->l[k] = v.l[k];
}

}  // namespace bgv
