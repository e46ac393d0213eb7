// The pubkey gather (k_pk_chunk) in its own translation unit, compiled with
// the Fp product INLINED (BGV_FPMUL_CALL=0).  Every call to the product leaf
// of the other units begins with s_waitcnt vmcnt(0) (the AMDGPU function
// prologue), so a table row loaded ahead would be waited for at the next
// product; inlined, the next row's 96 bytes stay in flight while this row's
// mixed addition runs.  The gather is bound by the latency of random rows:
// 12.98 M of them per C4 segment.
#define BGV_FPMUL_CALL 0
#ifndef BGV_FP2_INLINE
#define BGV_FP2_INLINE 1
#endif
#ifndef BGV_POINT_INLINE
#define BGV_POINT_INLINE 1
#endif
#include "bgv_internal.h"

namespace bgv {

#ifndef BGV_PKC_WAVES
#define BGV_PKC_WAVES 2
#endif

// PublicKey.aggregate (chain/bls/utils.ts:11) as a balanced gather: every
// set's index list is cut into chunks of PK_CHUNK keys (a 512-key
// sync-committee set is 16 chunks, a 128-key attestation 4, a single 1) so
// lanes of one wave do equal work; chunk offsets come from a device scan
// (bgv_kernels.hip k_chunk_count / k_scan / k_chunk_set).  Offsets that run
// backwards give the set no chunks, and the chunk scan is clipped at
// chunk_bound: no access leaves the buffers.
__global__ void __launch_bounds__(64, BGV_PKC_WAVES) k_pk_chunk(dev_batch b, dev_work w) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= min(w.chunk_off[b.n_sets], b.chunk_bound)) return;
  const uint32_t i = w.chunk_set[g];
  const uint32_t beg = b.pk_off[i] + (g - w.chunk_off[i]) * PK_CHUNK;
  const uint32_t end = min(beg + PK_CHUNK, b.pk_off[i + 1]);
  g1j acc;
  jac_set_inf(acc);
  bool range_err = false;
  // software pipelined: the next row is loaded before this row is added
  g1a nxt;
  if (beg < end) load_pk(nxt, b, b.pk_idx[beg], range_err);
  for (uint32_t k = beg; k < end; k++) {
    const g1a p = nxt;
    if (k + 1 < end) load_pk(nxt, b, b.pk_idx[k + 1], range_err);
    if (g1a_is_zero(p)) continue;  // infinity entry adds nothing
    jac_add_aff(acc, acc, p);
  }
  if (range_err) {  // marker (X, Y, Z) = (0, 1, 1): not on E1, never produced by point additions
    fp_set_zero(acc.x);
    acc.y = FP_ONE;
    acc.z = FP_ONE;
  }
  w.pk_part[g] = acc;
}

void launch_pk_gather(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.chunk_bound) hipLaunchKernelGGL(k_pk_chunk, dim3((b.chunk_bound + 63u) / 64u), dim3(64), 0, st, b, w);
}

}  // namespace bgv
