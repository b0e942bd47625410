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

#endif
