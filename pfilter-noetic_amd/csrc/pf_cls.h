// The BPF front end on the device: groundSeg::ground_seg (include/preProcess.hpp:398-505) and
// nongroundExtract::featureExtract (:646-689), as src/additionNode.cpp:21-45 chains them.
//
//   ground_seg     k_gs_bounds   x/y bounds (ordered-int atomics); the last workgroup sizes the 2-D
//                                grid (row, col in double, :412-415) and clears its cells
//                  k_gs_assign   per point: cell id, count, lowest z in (min, max ground height]
//                  k_gs_nbmin    per cell: 3x3 minimum of the lowest z (interior cells, :451-467)
//                  k_gs_keys     per point: sort key reproducing the reference's push order
//                                (0 = above max height, pushed first in input order; 1 + cell =
//                                non-ground of that cell; 2^15 + cell = ground; 0xFFFF = dropped)
//                  radix sort (16-bit keys, stable) + k_gs_gather -> the non-ground cloud U
//   featureExtract grid_build    1 m cell grid over U (pf_knn.h)
//                  k_cls_pca     per U point: the <= k nearest U points with d^2 < r^2 (a team of 16
//                                lanes keeps the sorted top-k in LDS), PCA, the class decision
//                  radix sort by class (stable) + k_cls_out -> beam / pillar / facade clouds in U order
#pragma once
#include "pf_common.h"
#include "pf_dcvc.h"
#include "pf_knn.h"
#include "pf_prims.h"

namespace pf {

constexpr int kClsMaxK = 32;                 // neighbour_k limit (LDS top-k list)
constexpr int kGsMaxCells = (1 << 15) - 2;   // ground grid cells (keys must stay below 0xFFFF)

enum ClsCounter {
    CC_N = 0,        // input points
    CC_NU,           // non-ground points (U)
    CC_NG,           // ground points
    CC_CLS,          // [4] class sizes in key order: beam, pillar, facade, none
    CC_ERR = CC_CLS + 4,   // 1: ground grid larger than kGsMaxCells
    CC_NUG,          // ground_seg's non-ground count (CC_NU after DCVC, when it runs, is its output's)
    CC_COUNT
};

struct ClsGPU {
    pf_cls_params prm{};
    size_t cap = 0;
    int* cnt = nullptr;          // [CC_COUNT]
    u32* gb = nullptr;           // [4] ordered-float bounds min x, min y, max x, max y (+ arrival)
    int* gdim = nullptr;         // [4] row, col, num_grid, valid
    u32* cell_cnt = nullptr;     // [kGsMaxCells]
    u32* cell_minz = nullptr;    // [kGsMaxCells] ordered float
    float* cell_nb = nullptr;    // [kGsMaxCells]
    u32* pcell = nullptr;        // [cap] ground cell of each input point (or ~0)
    u32* keys = nullptr;         // [cap]
    u32* vals = nullptr;         // [cap] after the sort: U index -> input index
    float4* pts = nullptr;       // [cap] staging of host scans
    float4* U = nullptr;         // [cap] non-ground cloud
    u32* ckeys = nullptr;        // [cap] class key per U point
    u32* cvals = nullptr;        // [cap]
    uint8_t* code = nullptr;     // [cap] index_with_feature code per U point
    int* ptnum = nullptr;        // [cap] neighbours found per U point
    int* idx_out = nullptr;      // [cap] input indices of beam | pillar | facade
    float4* box = nullptr;       // [2 * (cap / 16 + 1)] bounding box (lo, hi) of every 16-point chunk
    float4* nrm = nullptr;       // [cap] per U point: the normal assign_normal writes (preProcess.hpp:327-346)
    u32* nbr = nullptr;          // [cap * kClsMaxK] neighbour lists (U indices, ascending distance)
    GridGPU grid;
    PrimWork w;
    int* sticky = nullptr;       // not owned: where CC_ERR is also latched (OdomGPU::errw)
    DcvcGPU* dcvc = nullptr;     // curvedfilter (pf_cls_set_dcvc / pf_bpf_set_dcvc); null: off
    float4* dU = nullptr;        // [cap] DCVC output staging
    u32* dV = nullptr;           // [cap]
};
// curvedfilter on / off (p null); allocates the DCVC state on first use
int cls_set_dcvc(ClsGPU& c, const pf_dcvc_params* p);

int cls_alloc(ClsGPU& c, size_t cap);
void cls_free(ClsGPU& c);

// Enqueue the chain on s for d_pts[0 .. *d_n). out / out_cnt (optional, may be null): the beam,
// pillar and facade clouds as float4 (x, y, z, 0) and their device-resident sizes. idx: also write
// the input indices of the three classes (c.idx_out) and of the ground points (c.keys region after
// U, see cls_ground_offset).
// ground_only: stop after ground_seg (c.vals: non-ground then ground input indices).
void cls_enqueue(ClsGPU& c, const float4* d_pts, const int* d_n, float4* const* out, int* const* out_cnt,
                 bool idx, hipStream_t s, bool ground_only = false);

}  // namespace pf
