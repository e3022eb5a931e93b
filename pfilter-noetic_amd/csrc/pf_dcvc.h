// curvedVoxel (DCVC, Dynamic Curved-Voxel Clustering; src/additionClass.cpp:1-497) on the device: the
// filter src/additionNode.cpp:29-39 puts between ground_seg and featureExtract (curvedfilter, on in
// launch/pfilter_kitti.launch:8).
//
//   k_dc_polar    per point: range, pitch, azimuth in double (convertToPolar :85-136, out-of-range
//                 points kept at (0, 0, 0)); ordered-bits atomics for max range / min, max pitch; the
//                 last workgroup forms width, height and the polar bounds (the reference's while loop,
//                 sequential doubles) and counts the call (the first call starts the range at 5 m)
//   k_dc_keys     per point: polar / pitch / azimuth index and voxel index (createHashTable :143-177)
//   radix sort    (voxel, point) stable, segments = voxels
//   k_dc_voxels   per voxel: key, point count; its slot entered in a dense table over the voxel index
//                 space (cleared again by k_dc_compress), so a neighbour lookup is one load
//   k_dc_link     per voxel: its <= 27 search positions (searchKNN :196-225 with its azimuth wrap /
//                 clamp and pitch-layer quirks) looked up at once; parent = the smallest (ECL-CC style
//                 first link), the other edges listed (a two-way edge at its smaller end only)
//   k_dc_union    per voxel: union over its listed edges (lock-free union-find: smaller root wins,
//                 path halving)
//   k_dc_compress per voxel: full compression, its component's point count and first point (one atomic
//                 pair per distinct root and wave), the voxel table emptied
//   k_dc_rank     one workgroup: components larger than minSeg ranked by size, then first point
//   k_dc_label    per voxel: its points' sort keys (component rank or dropped), then a stable sort by
//                 rank gives the published order (labelAnalysis :325-355, colorSegmentation :360-372)
//
// The reference's loops run under OpenMP with shared temporaries, so its clusters are not a function
// of its input; its serial reading (oracle/pfref_dcvc.cpp) leaves some neighbours of a processed point
// unlabelled (a greedy pass), which no parallel formulation reproduces. The device computes the
// connected components of the same voxel neighbourhood relation — bit-exact against the oracle's
// component mode — and is held to the serial reading statistically (tests/test_gpu_dcvc.py).
#pragma once
#include "pf_common.h"
#include "pf_prims.h"

namespace pf {

constexpr int kDcMaxBounds = 4096;      // polar bounds (rings of the curved grid)
constexpr int kDcMaxClusters = 4096;    // kept components (each > minSeg points)
// DcvcGPU::dim slots
enum { D_POLAR = 0, D_WIDTH, D_HEIGHT, D_CALLS, D_ERR, D_NCLUST, D_NKEPT, D_N };

struct DcvcGPU {
    pf_dcvc_params prm{};
    size_t cap = 0;
    u64* red = nullptr;          // [8] ordered bits: max range, min pitch, max pitch; [3] arrival; [4] min range
    double* bounds = nullptr;    // [kDcMaxBounds]
    int* dim = nullptr;          // [8] polarNum, width, height, calls, err, nvox, nkept, n
    double4* pol = nullptr;      // [cap] range, pitch, azimuth
    u32* keys = nullptr;         // [cap]
    u32* vals = nullptr;         // [cap]
    u32* segstart = nullptr;     // [cap + 1]
    int* seg_aux = nullptr;      // [8] segment counts (nseg, nlt[3], nvalid)
    u32* parent = nullptr;       // [cap] union-find over voxels
    u32* csize = nullptr;        // [cap] component point count (at the root)
    u32* cfirst = nullptr;       // [cap] component first point (at the root)
    u32* crank = nullptr;        // [cap] rank + 1 of a kept root, 0 otherwise
    u32* okeys = nullptr;        // [cap] per point: rank (published order) or 0xFFFFFFFF
    u32* ovals = nullptr;        // [cap] after the last sort: the kept points in the published order
    u32* plab = nullptr;         // [cap] per point: its component's rank + 1, or 0 (dropped)
    u32* ukey = nullptr;         // [cap] per voxel: its key
    u32* ucount = nullptr;       // [cap] per voxel: its point count
    int* vtab = nullptr;         // [vtab_cells] voxel slot of every cell of the index space, -1 empty
    long long vtab_cells = 0;    // (0: the index space is too large, voxels are found by binary search)
    u32* edges = nullptr;        // [cap][26] per voxel: the search edges it unions (k_dc_link)
    u32* ecount = nullptr;       // [cap]
    PrimWork w;
};

int dcvc_alloc(DcvcGPU& d, size_t cap);
// the parameters, and the voxel table sized for their index space (allocated outside any capture)
int dcvc_set_params(DcvcGPU& d, const pf_dcvc_params& p);
void dcvc_free(DcvcGPU& d);
// the call counter back to 0 (the next call is a first frame)
int dcvc_reset(DcvcGPU& d, hipStream_t s);
// as after one call: the next run is not the first (its range bounds start from 0, not the member
// defaults); the second front-end lane of a BPF handle (pf_odom.h OdomGPU::front2)
int dcvc_mark_called(DcvcGPU& d, hipStream_t s);
// the parameter check of pf_dcvc_create: positive steps and a ring width start_r - k delta_r that
// stays positive up to max_range within the bound table (else a frame would overflow it)
bool dcvc_params_valid(const pf_dcvc_params* p);

// DCVC of pts[0 .. *d_n) (float4 x, y, z, any). Result: kept point indices in the published order at
// *out_idx (device, dim[D_NKEPT] of them), per point label in plab. Enqueued on s, no host round trip.
void dcvc_enqueue(DcvcGPU& d, const float4* pts, const int* d_n, hipStream_t s, u32** out_idx);

}  // namespace pf
