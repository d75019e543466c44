// Host-side coverage check of tile_order.h (tests/test_tile_order.py builds and runs it on CPU):
// for every partition size (1/2/4/8 XCDs), order mode and a set of tile grids, the workgroup → tile
// map must hit every tile exactly once, and the SPX super-block order must give each XCD a 4×8
// corner per round.  Prints "tile order OK" or the first violation.
#include <cstdio>
#include <vector>

#include "tile_order.h"

int main() {
  const int grids[][2] = {{32, 16}, {9, 5}, {16, 16}, {48, 32}, {4, 8}, {8, 8}, {1, 1}, {64, 64}};
  for (int lx = 0; lx < 4; ++lx) {
    const int x = 1 << lx, xn = x >= 2 ? 2 : 1, sbm = 4 * (x / xn), sbn = 8 * xn;
    for (const auto& g : grids) {
      const int tm = g[0], tn = g[1];
      const bool fits = tm % sbm == 0 && tn % sbn == 0;
      for (int mode = 0; mode < 3; ++mode) {
        if ((mode && !fits) || (mode == 2 && x != 8)) continue;
        std::vector<int> seen(tm * tn, 0);
        for (int b = 0; b < tm * tn; ++b) {
          int m = -1, n = -1;
          amdk8s::block_tile(b, tm, tn, lx | (mode << 2), 8, m, n);
          if (m < 0 || m >= tm || n < 0 || n >= tn || seen[m * tn + n]++) {
            std::printf("FAIL: xcds %d mode %d grid %dx%d block %d -> (%d, %d)\n", x, mode, tm, tn, b, m, n);
            return 1;
          }
        }
        if (mode == 1) {  // each XCD's 32 concurrent tiles form one 4(M)x8(N) corner
          for (int xcd = 0; xcd < x; ++xcd) {
            int mlo = 1 << 30, mhi = -1, nlo = 1 << 30, nhi = -1;
            for (int j = 0; j < 32; ++j) {
              int m, n;
              amdk8s::block_tile(j * x + xcd, tm, tn, lx | (1 << 2), 8, m, n);
              mlo = m < mlo ? m : mlo; mhi = m > mhi ? m : mhi;
              nlo = n < nlo ? n : nlo; nhi = n > nhi ? n : nhi;
            }
            if (mhi - mlo != 3 || nhi - nlo != 7) {
              std::printf("FAIL: xcds %d grid %dx%d xcd %d corner %dx%d\n", x, tm, tn, xcd,
                          mhi - mlo + 1, nhi - nlo + 1);
              return 1;
            }
          }
        }
      }
    }
  }
  std::printf("tile order OK\n");
  return 0;
}
