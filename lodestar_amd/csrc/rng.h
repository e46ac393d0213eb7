// Batch scalars drawn on the device: ChaCha20 (RFC 8439 section 2.3 block
// function) keyed by 32 bytes of host getrandom() per call.  Set i takes the
// first 8 bytes of block (counter = i) that are non-zero as its 64-bit
// multiplier r_i, the role of blst's per-set random scalars in
// verifyMultipleSignatures (reached from chain/bls/maybeBatch.ts:18-25).
// Drawing them here removes an 800 KB host getrandom() + copy from every C4
// call.
#pragma once
#include "bls_types.h"

namespace bgv {

BGV_HD uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

BGV_HD void chacha_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  a += b; d ^= a; d = rotl32(d, 16);
  c += d; b ^= c; b = rotl32(b, 12);
  a += b; d ^= a; d = rotl32(d, 8);
  c += d; b ^= c; b = rotl32(b, 7);
}

// out = ChaCha20 block(key, counter, nonce) as 16 little-endian words
BGV_HD void chacha20_block(uint32_t out[16], const uint32_t key[8], uint32_t counter, const uint32_t nonce[3]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4], key[5], key[6], key[7], counter, nonce[0], nonce[1], nonce[2]};
  uint32_t x[16];
  for (int i = 0; i < 16; i++) x[i] = s[i];
  for (int r = 0; r < 10; r++) {
    chacha_qr(x[0], x[4], x[8], x[12]);
    chacha_qr(x[1], x[5], x[9], x[13]);
    chacha_qr(x[2], x[6], x[10], x[14]);
    chacha_qr(x[3], x[7], x[11], x[15]);
    chacha_qr(x[0], x[5], x[10], x[15]);
    chacha_qr(x[1], x[6], x[11], x[12]);
    chacha_qr(x[2], x[7], x[8], x[13]);
    chacha_qr(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

// r_i: first non-zero 64-bit word of block i (an all-zero block, probability
// 2^-512, would yield 1)
BGV_HD uint64_t batch_scalar(const uint32_t key[8], uint32_t i, const uint32_t nonce[3]) {
  uint32_t blk[16];
  chacha20_block(blk, key, i, nonce);
  for (int k = 0; k < 8; k++) {
    const uint64_t v = (uint64_t)blk[2 * k] | ((uint64_t)blk[2 * k + 1] << 32);
    if (v) return v;
  }
  return 1;
}

}  // namespace bgv
