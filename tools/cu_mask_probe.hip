// Where do the workgroups of a CU-masked stream run?  For each mask layout the
// probe launches 8,192 one-wave workgroups on a stream made by
// hipExtStreamCreateWithCUMask; every workgroup reads its XCC (HW_REG_XCC_ID)
// and its SE / SH / CU (HW_REG_HW_ID) and writes them with a vector store.
// The host prints, per layout, how many distinct CUs ran work on each XCC.
//   hipcc --offload-arch=gfx950 -O2 tools/cu_mask_probe.hip -o tools/cu_mask_probe && ./tools/cu_mask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void probe(uint32_t* out) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // keep the wave resident a little so the dispatcher spreads the grid
  uint32_t v = threadIdx.x;
  for (int i = 0; i < 20000; i++) v = v * 1664525u + 1013904223u;
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc | (v & 0x80000000u ? 0x100u : 0u) ;
  }
}

int main() {
  int n_cu = 0;
  CHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  const int words = (n_cu + 31) / 32;
  const int blocks = 8192;
  uint32_t* d;
  CHK(hipMalloc(&d, 2 * blocks * sizeof(uint32_t)));
  std::vector<uint32_t> h(2 * blocks);
  struct layout { std::string name; std::vector<int> ids; };
  std::vector<layout> ls;
  auto range = [](int a, int b) { std::vector<int> v; for (int i = a; i < b; i++) v.push_back(i); return v; };
  ls.push_back({"all", range(0, n_cu)});
  ls.push_back({"top8 (248-255)", range(n_cu - 8, n_cu)});
  ls.push_back({"low8 (0-7)", range(0, 8)});
  { std::vector<int> v; for (int k = 0; k < 8; k++) v.push_back(32 * k + 31); ls.push_back({"32k+31", v}); }
  { std::vector<int> v; for (int k = 0; k < 8; k++) v.push_back(n_cu - 64 + 8 * k + 7); ls.push_back({"8k+7 top", v}); }
  ls.push_back({"ids 0-31", range(0, 32)});
  { std::vector<int> v; for (int k = 0; k < 32; k++) v.push_back(8 * k); ls.push_back({"8k", v}); }
  for (int single : {0, 1, 2, 3, 4, 5, 6, 7, 8, 16, 32, 64, 128, 255}) ls.push_back({"id " + std::to_string(single), {single}});
  for (auto& L : ls) {
    std::vector<uint32_t> mask(words, 0u);
    for (int id : L.ids) mask[id / 32] |= 1u << (id % 32);
    hipStream_t s;
    CHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask.data()));
    CHK(hipMemsetAsync(d, 0xff, 2 * blocks * sizeof(uint32_t), s));
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, s, d);
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpy(h.data(), d, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    CHK(hipStreamDestroy(s));
    std::map<int, std::set<int>> per_xcc;  // xcc -> {se*64 + sh*16 + cu}
    for (int b = 0; b < blocks; b++) {
      const uint32_t hw = h[2 * b], x = h[2 * b + 1] & 0xf;
      const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      per_xcc[x].insert(se * 64 + sh * 16 + cu);
    }
    printf("%-16s ids=%3zu  xccs=%zu:", L.name.c_str(), L.ids.size(), per_xcc.size());
    for (auto& [x, cus] : per_xcc) {
      printf("  x%d:%zu[", x, cus.size());
      int shown = 0;
      for (int c : cus) { if (shown++ < 4) printf("%s%d.%d.%d", shown > 1 ? " " : "", c / 64, (c / 16) % 4, c % 16); }
      printf("%s]", cus.size() > 4 ? " .." : "");
    }
    printf("\n");
  }
  CHK(hipFree(d));
  return 0;
}
