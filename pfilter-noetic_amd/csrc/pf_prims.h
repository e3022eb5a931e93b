// Device-wide primitives with device-resident element counts (no host round trip).
#pragma once
#include "pf_common.h"

namespace pf {

constexpr int kSortMaxBlocks = 256;   // max workgroups of the sort / scan grids
constexpr int kSortTile = 2048;       // keys per tile (256 threads x 8)

struct PrimWork {
    u32* keys_tmp = nullptr;   // cap
    u32* vals_tmp = nullptr;   // cap
    u32* bhist = nullptr;      // [4 passes][256] global digit counts (zero between sorts)
    u64* status = nullptr;     // [4 passes][max_tiles][256] look-back words
    u32* tickets = nullptr;    // [8]: [4] histogram arrivals, [5] scan arrivals
    u32* dbase = nullptr;      // [4 passes][256] exclusive digit bases
    u64* scan_status = nullptr;// [max_tiles] scan look-back words (zero between calls)
    int* err = nullptr;        // look-back spin limit hit (never expected)
    size_t cap = 0, max_tiles = 0, scan_tiles = 0;
};

// cap: largest sort; scan_cap: largest scan (defaults to cap)
int prim_alloc(PrimWork& w, size_t cap, size_t scan_cap = 0);
void prim_free(PrimWork& w);

// Stable sort of (keys, vals)[0 .. *d_n) by the low `bits` bits of keys (8-bit digits). With kout/vout
// null the pass count is rounded up to even so the result is back in keys/vals; otherwise *kout/*vout
// name the buffers holding the result (keys/vals or the PrimWork scratch).
void radix_sort_pairs(u32* keys, u32* vals, const int* d_n, int bits, PrimWork& w, hipStream_t s,
                      u32** kout = nullptr, u32** vout = nullptr);

// Segments of stably sorted keys (bit 31 = cloud id, 0xFFFFFFFF = dropped entries, sorted last):
// segstart[s] = first index of segment s; *d_nseg = number of segments; *d_nseg_c0 = segments of
// cloud 0; *d_nvalid = number of non-sentinel keys.
void segment_starts(const u32* keys, const int* d_n, u32* segstart, int* d_nseg, int* d_nseg_c0, int* d_nvalid,
                    PrimWork& w, hipStream_t s);

// out[i] = sum(in[0..i)) for i < *d_n; *d_total = sum(in[0..n)) when d_total != nullptr.
void scan_exclusive(const u32* in, u32* out, const int* d_n, u32* d_total, PrimWork& w, hipStream_t s);

}  // namespace pf
