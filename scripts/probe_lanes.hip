// Probe of gfx950 cross-lane primitives (DPP controls, permlane16/32_swap): prints, for each,
// the source lane every lane receives.  Dev tool (not part of libgmp).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
  const int l = threadIdx.x;
  int v = l;
  out[0 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x128, 0xF, 0xF, false);  // row_ror:8
  out[1 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  out[2 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x4E, 0xF, 0xF, false);   // quad_perm 2301
  out[3 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0xB1, 0xF, 0xF, false);   // quad_perm 1032
  out[4 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  out[5 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  out[6 * 64 + l] = a[0];
  out[7 * 64 + l] = a[1];
  auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  out[8 * 64 + l] = b[0];
  out[9 * 64 + l] = b[1];
  out[10 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x140, 0xF, 0xF, false);  // row_mirror
  out[11 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xF, 0xF, true);  // row_shr:1 bc
}

int main() {
  int* d;
  hipMalloc(&d, 12 * 64 * sizeof(int));
  probe<<<1, 64>>>(d);
  int h[12 * 64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[12] = {"row_ror8", "row_half_mirror", "qp2301", "qp1032", "row_shr1",
                           "row_shr8", "pl32swap.0", "pl32swap.1", "pl16swap.0", "pl16swap.1",
                           "row_mirror", "row_shr1_bc"};
  for (int k = 0; k < 12; ++k) {
    printf("%-16s", names[k]);
    for (int l = 0; l < 64; ++l) printf(" %d", h[k * 64 + l]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
