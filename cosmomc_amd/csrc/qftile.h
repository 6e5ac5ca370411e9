// Device pieces of the f64-MFMA quadratic form shared by its kernels
// (quadform.hip) and by the sampler's unified step launch (mh_step_kernel): the
// swizzled LDS operand tiles, their LDS-DMA fill and the XCD-aware
// workgroup -> (item, walker tile) placement.
#pragma once

#include "quadform.h"

namespace cmamd {

static constexpr int BK = 32;            // k depth staged per pipeline step (16 chunks of 16 B per row)

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// LDS image of a 64-row x BK-double operand tile: rows of 256 B, unpadded;
// the 16-byte chunk c of row r lives at physical chunk c ^ swz(r).  The
// swizzle makes both the LDS-DMA fill (linear 1 KB pieces) and the MFMA
// fragment reads (ds_read_b128, 8 consecutive k per lane) bank-conflict free.
__device__ __forceinline__ int swz(int r) { return ((r >> 2) & 3) | ((r & 3) << 2); }

// Fill one 64 x BK tile: rows row0..row0+63 of a row-major matrix (stride ld
// doubles), columns k0..k0+BK-1.  4 waves x 4 instructions of 1 KB; lane l
// of instruction j writes LDS bytes [l*16, l*16+16) of piece j = physical
// chunk (l & 15) of row 4j + (l >> 4), so it loads the logical chunk
// (l & 15) ^ swz(row) from global memory.
__device__ __forceinline__ void dma_tile(double *lds_tile, const double *g, size_t ld, int k0, int wave, int lane)
{
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int piece = wave * 4 + q;                 // 0..15, 4 rows each
        const int r = piece * 4 + (lane >> 4);
        const int lc = (lane & 15) ^ swz(r);
        const double *src = g + (size_t)r * ld + k0 + lc * 2;
        __builtin_amdgcn_global_load_lds((gbl_void_t *)src, (lds_void_t *)(lds_tile + piece * 4 * BK), 16, 0, 0);
    }
}

static constexpr int QF_LDS_DOUBLES = 2 * 2 * QF_TILE * BK;   // [buf][A|B][64][BK], 64 KB

// Workgroup b of the launch (b = item + tile * n_items in launch order) ->
// its (item, walker tile).  XCD-aware placement: blocks b and b+8 share an
// XCD; give each XCD whole walker tiles so a tile's Delta stays in one L2
// (speed only)
__device__ __forceinline__ void qf_place(int b, int n_items, int xcd_map, int &item_ix, int &tile) {
    if (xcd_map) {
        const int x = b & 7, j = b >> 3;
        tile = x + 8 * (j / n_items);
        item_ix = j % n_items;
    } else {
        item_ix = b % n_items;
        tile = b / n_items;
    }
}

}  // namespace cmamd
