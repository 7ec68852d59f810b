// mfma_probe.hip -- checks the operand/result lane maps of
// v_mfma_i32_16x16x64_i8 on gfx950 with exact integer data (dev tool).
//
// Hypothesis used by the MFMA transform passes: lane l holds 16 bytes of A
// for row (l & 15) and 16 bytes of B for column (l & 15), the two sharing
// one set of K indices per lane group g = l >> 4 (whatever their order), and
// D holds column (l & 15), rows 4 g + i in register i.  Then
//   D[row][col] = sum_{g, j} A_lane(16 g + row)[j] * B_lane(16 g + col)[j].
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_probe.hip -o tools/bin/mfma_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_probe(const int* a, const int* b, int* d) {
  const int l = threadIdx.x;
  v4i A, B, C = {0, 0, 0, 0};
  for (int r = 0; r < 4; ++r) {
    A[r] = a[l * 4 + r];
    B[r] = b[l * 4 + r];
  }
  const v4i D = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, C, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = D[r];
}

int main() {
  int ha[256], hb[256], hd[256];
  srand(12345);
  for (int i = 0; i < 256; ++i) {
    ha[i] = (rand() << 16) ^ rand();
    hb[i] = (rand() << 16) ^ rand();
  }
  // extremes in one lane: all -128 bytes
  ha[0] = ha[1] = ha[2] = ha[3] = (int)0x80808080u;
  hb[0] = hb[1] = hb[2] = hb[3] = (int)0x80808080u;
  int *da, *db, *dd;
  if (hipMalloc(&da, 1024) || hipMalloc(&db, 1024) || hipMalloc(&dd, 1024)) return 2;
  (void)hipMemcpy(da, ha, 1024, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, da, db, dd);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  (void)hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int row = 0; row < 16; ++row)
    for (int col = 0; col < 16; ++col) {
      long s = 0;
      for (int g = 0; g < 4; ++g) {
        const signed char* ab = (const signed char*)&ha[(16 * g + row) * 4];
        const signed char* bb = (const signed char*)&hb[(16 * g + col) * 4];
        for (int j = 0; j < 16; ++j) s += (long)ab[j] * bb[j];
      }
      const int lane = 16 * (row >> 2) + col, reg = row & 3;
      if (hd[lane * 4 + reg] != (int)s) {
        if (bad < 8) printf("mismatch row %d col %d: got %d want %ld\n", row, col, hd[lane * 4 + reg], s);
        ++bad;
      }
    }
  printf("mfma_i32_16x16x64_i8 lane-map hypothesis: %s (%d mismatches of 256)\n", bad ? "FAILED" : "OK", bad);
  return bad ? 1 : 0;
}
