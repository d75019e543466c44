// Workgroup → 256×256 output-tile order for the MFMA GEMMs, for any MI355X compute partition.
//
// The dispatcher places workgroup b on XCD (b mod X), X = XCDs in the partition the kernel runs on:
// 8 in SPX (256 CUs), 4 in DPX, 2 in QPX, 1 in CPX (32 CUs: each CPX partition is one XCD with its
// own 4 MiB L2 — the "8 concurrent pods × 1 partition" case of BASELINE.json config 5).  Each XCD
// runs 32 tiles at once (one per CU), so the order gives every XCD a 4(M)×8(N) corner of a
// super-block of X·32 tiles: the corner's A and B panels are shared inside that XCD's L2, and the
// super-block's panels stay in the 256 MiB Infinity Cache.  Super-blocks are walked in snake order so
// consecutive rounds share a panel set.  When the tile grid is not a whole number of super-blocks,
// GROUP_M-grouped order over the XCD-contiguous remap is used instead.
//
// Super-block shape per partition (corners arranged xm × xn, xn = 2 when X ≥ 2):
//   X = 8: 16×16 tiles (4×2 corners, the SPX order measured in docs/gemm_tuning.md)
//   X = 4:  8×16        X = 2: 8×8        X = 1: 4×8
//
// The kernels take one `order` argument: bits 0-1 = log2(X), bits 2-3 = super-block mode
// (0 = GROUP_M order, 1 = 4×8 corners, 2 = 8×4 corners — an SPX-only A/B knob).
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>

namespace amdk8s {

// XCDs of the partition the current device is (AMDK8S_GEMM_XCDS=1|2|4|8 overrides, for tests and
// A/B runs of the orders on an SPX device).
inline int partition_xcds() {
  if (const char* e = getenv("AMDK8S_GEMM_XCDS")) {
    const int x = atoi(e);
    if (x == 1 || x == 2 || x == 4 || x == 8) return x;
  }
  static int cache[64];  // per device; 0 = not queried yet
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 8;
  if (dev >= 0 && dev < 64 && cache[dev]) return cache[dev];
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  int x = (cus + 16) / 32;  // 32 CUs per XCD on MI355X
  x = x >= 8 ? 8 : x >= 4 ? 4 : x >= 2 ? 2 : 1;
  if (dev >= 0 && dev < 64) cache[dev] = x;
  return x;
}

// Host: the kernels' `order` argument for a tiles_m × tiles_n grid.  AMDK8S_W4_SUPERBLOCK=0 forces
// GROUP_M order, =2 the 8×4 corners (SPX only).
inline int tile_order_arg(int tiles_m, int tiles_n) {
  const int x = partition_xcds();
  const int lx = x == 8 ? 3 : x == 4 ? 2 : x == 2 ? 1 : 0;
  const int xn = x >= 2 ? 2 : 1, xm = x / xn;
  const int sbm = 4 * xm, sbn = 8 * xn;
  const char* e = getenv("AMDK8S_W4_SUPERBLOCK");
  int mode = (tiles_m % sbm == 0 && tiles_n % sbn == 0) ? 1 : 0;
  if (e && e[0] == '0') mode = 0;
  if (mode && e && e[0] == '2' && x == 8) mode = 2;
  return lx | (mode << 2);
}

// Tile coordinates (in tiles) of workgroup `bid` (host-callable for the coverage test).
__host__ __device__ __forceinline__ void block_tile(int bid, int tiles_m, int tiles_n, int order,
                                                    int group_m, int& tm, int& tn) {
  const int lx = order & 3, mode = (order >> 2) & 3;
  const int x = 1 << lx;
  const int xcd = bid & (x - 1);
  const int i = bid >> lx;
  if (mode) {
    const int xn = x >= 2 ? 2 : 1;
    const int sbm_t = 4 * (x / xn), sbn_t = 8 * xn;  // super-block size in tiles
    const int round = i >> 5, j = i & 31;
    const int sb_n_count = tiles_n / sbn_t;
    const int sbm = round / sb_n_count;
    int sbn = round - sbm * sb_n_count;
    if (sbm & 1) sbn = sb_n_count - 1 - sbn;
    if (mode == 2) {  // SPX, 8(M)×4(N) corners
      tm = sbm * 16 + (xcd & 1) * 8 + (j & 7);
      tn = sbn * 16 + (xcd >> 1) * 4 + (j >> 3);
    } else {
      tm = sbm * sbm_t + (xcd / xn) * 4 + (j & 3);
      tn = sbn * sbn_t + (xcd % xn) * 8 + (j >> 2);
    }
  } else {
    const int nwg = tiles_m * tiles_n;
    const int q = nwg >> lx, r = nwg & (x - 1);
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
    const int group = wgid / (group_m * tiles_n);
    const int first_m = group * group_m;
    const int gsz = min(tiles_m - first_m, group_m);
    const int in_group = wgid - group * group_m * tiles_n;
    tm = first_m + in_group % gsz;
    tn = in_group / gsz;
  }
}

}  // namespace amdk8s
