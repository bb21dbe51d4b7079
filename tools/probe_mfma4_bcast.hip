// Probe: v_mfma_f64_4x4x4_4b with the A-broadcast modifiers (cbsz = 2: the A
// operand of block abid is used by all four blocks).  Lane l = 16 X + 4 b + Y
// supplies A[m=Y][k=X], B[k=X][n=Y] of block b and receives D[m=X][n=Y]
// (tools/probe_mfma4.hip).  Prints the max deviation from that model.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mfma4_bcast.hip -o tools/probe_mfma4_bcast
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

template <int ABID>
__global__ void k_probe(const double *a, const double *b, double *d) {
  const int l = threadIdx.x;
  d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, ABID, 0);
}
__global__ void k_plain(const double *a, const double *b, double *d) {
  const int l = threadIdx.x;
  d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 0, 0, 0);
}

int main() {
  double ha[64], hb[64], hd[64], *da, *db, *dd;
  for (int l = 0; l < 64; ++l) {
    ha[l] = 1.0 + l * 0.37 - (l % 5) * 1.1;
    hb[l] = 0.5 - l * 0.11 + (l % 7) * 0.3;
  }
  (void)hipMalloc(&da, 512);
  (void)hipMalloc(&db, 512);
  (void)hipMalloc(&dd, 512);
  (void)hipMemcpy(da, ha, 512, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, 512, hipMemcpyHostToDevice);
  {
    k_plain<<<1, 64>>>(da, db, dd);
    (void)hipMemcpy(hd, dd, 512, hipMemcpyDeviceToHost);
    double e = 0.0;
    for (int X = 0; X < 4; ++X)
      for (int bb = 0; bb < 4; ++bb)
        for (int Y = 0; Y < 4; ++Y) {
          double s0 = 0.0;
          for (int k = 0; k < 4; ++k) s0 += ha[16 * k + 4 * bb + X] * hb[16 * k + 4 * bb + Y];
          e = fmax(e, fabs(hd[16 * X + 4 * bb + Y] - s0));
        }
    printf("cbsz=0: max |D - plain model| = %.3e\n", e);
    // which A lanes feed block bb's D: fit D against A lane sets
    for (int bb = 0; bb < 4; ++bb) printf("D block %d lane0 %.6f\n", bb, hd[4 * bb]);
  }
  double worst = 0.0;
  for (int abid = 0; abid < 4; ++abid) {
    switch (abid) {
      case 0: k_probe<0><<<1, 64>>>(da, db, dd); break;
      case 1: k_probe<1><<<1, 64>>>(da, db, dd); break;
      case 2: k_probe<2><<<1, 64>>>(da, db, dd); break;
      default: k_probe<3><<<1, 64>>>(da, db, dd); break;
    }
    (void)hipMemcpy(hd, dd, 512, hipMemcpyDeviceToHost);
    double err = 0.0, err_nob = 0.0;
    for (int X = 0; X < 4; ++X)
      for (int bb = 0; bb < 4; ++bb)
        for (int Y = 0; Y < 4; ++Y) {
          // model: D[m=X][n=Y] of block bb = sum_k A_abid[m=X][k] B_bb[k][n=Y]
          double s = 0.0, s0 = 0.0;
          for (int k = 0; k < 4; ++k) {
            s += ha[16 * k + 4 * abid + X] * hb[16 * k + 4 * bb + Y];
            s0 += ha[16 * k + 4 * bb + X] * hb[16 * k + 4 * bb + Y];
          }
          err = fmax(err, fabs(hd[16 * X + 4 * bb + Y] - s));
          err_nob = fmax(err_nob, fabs(hd[16 * X + 4 * bb + Y] - s0));
        }
    printf("abid=%d: max |D - broadcast model| = %.3e, |D - no-broadcast model| = %.3e; D[0]=%.6f D[4]=%.6f\n", abid,
           err, err_nob, hd[0], hd[4]);
    worst = fmax(worst, err);
  }
  printf("%s\n", worst < 1e-12 ? "broadcast model holds" : "broadcast model FAILS");
  return 0;
}
