// tile_format.h -- the TILE backward's plan format constants, shared by the
// kernel (maxk_spgemm.hip) and the device plan builder (maxk_plan.hip); the
// Python side reads them through maxk_tile_format().
//
// A workgroup's distinct source rows are cut into chunks of kTileRows rows;
// chunk c is staged (LDS-DMA) into ring buffer c % kTileBufs of kTileBufRows
// rows, the last row of every buffer being a zero row for padding records.
// The DMA runs kTileBufs - 1 chunks ahead of the records.  Per (workgroup,
// wave) the header stream holds nch + kTileBufs - 1 int32x4 entries:
// e(i) = {counts of chunk i - (kTileBufs - 1) (0 for i < kTileBufs - 1),
//         source rows of the wave's three DMA pieces of chunk i}.
#ifndef MAXK_TILE_FORMAT_H
#define MAXK_TILE_FORMAT_H

#ifndef TILE_NBUF
#define TILE_NBUF 3
#endif
#ifndef TILE_BUF_ROWS
#define TILE_BUF_ROWS 48
#endif

// Record format: TILE_REC_WORDS = 2 -- {w = slot | staged row << 24, value}: the
// kernel derives the selector word, its bit offset and the row's LDS address
// from w with three scalar shifts per record; 4 -- {selector control word (byte
// 0: selector register index, byte 2: 4 + byte of it, bytes 1 / 3: 0x0c; the
// S2 operand of a v_perm_b32 that extracts the selector into byte 2), slot,
// LDS byte address of the staged row, value}: no scalar work besides the two
// register-index writes per record.
#ifndef TILE_REC_WORDS
#define TILE_REC_WORDS 4
#endif
constexpr int kTileRecWords = TILE_REC_WORDS;
static_assert(kTileRecWords == 2 || kTileRecWords == 4, "record words");

constexpr int kTileWaves = 16;
constexpr int kTileBufs = TILE_NBUF;
constexpr int kTileBufRows = TILE_BUF_ROWS;
constexpr int kTileRows = kTileBufRows - 1;
constexpr int kTilePieces = 3;  // DMA pieces (1 KB rows) per wave and chunk
static_assert(kTileWaves * kTilePieces >= kTileBufRows, "every buffer row has a DMA piece");
static_assert(kTileBufs >= 2 && kTileBufs * kTileBufRows <= 160, "ring fits the 160 KB of LDS");
static_assert((kTileBufs - 1) * kTileBufRows + kTileRows < 256, "row field of a record is 8 bits");

// Pieces (round 4): the (destination group g, source row r) space, x = g * V + r
// over G groups and V source rows, is cut into P equal ranges, one per
// workgroup b: [x_b, x_{b+1}) with x_b = ceil(b * G * V / P).  A workgroup
// whose range crosses a group boundary finishes one group's rows and starts the
// next group's.  The piece of (g, r) is p = g + b(x), b(x) = floor(x * P / (G * V)):
// ids 0 .. G + P - 2 (an id whose workgroup holds none of its group's rows has
// no edges).  Group g's pieces lie in workgroups b0(g) = floor(g * P / G) ..
// b1(g) = b((g + 1) * V - 1); piece b0 writes dXs, piece b0 + i partial plane
// i - 1 (summed into dXs afterwards, in plane order).  P = G * S cuts every
// group into S equal source ranges (the round-3 "splits").
__host__ __device__ inline int tile_wg_of(int64_t x, int64_t gv, int P)
{
    return (int)(x * P / gv);
}
__host__ __device__ inline int64_t tile_wg_start(int64_t b, int64_t gv, int P)
{
    return (b * gv + P - 1) / P;
}
__host__ __device__ inline int tile_piece(int g, int r, int V, int G, int P)
{
    const int64_t gv = (int64_t)G * V;
    return g + tile_wg_of((int64_t)g * V + r, gv, P);
}
// extra partial planes of group g (its pieces - 1)
__host__ __device__ inline int tile_group_planes(int g, int V, int G, int P)
{
    const int64_t gv = (int64_t)G * V;
    return tile_wg_of((int64_t)(g + 1) * V - 1, gv, P) - (int)((int64_t)g * P / G);
}

#endif
