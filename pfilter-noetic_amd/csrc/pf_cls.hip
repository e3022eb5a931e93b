// BPF front end kernels (see pf_cls.h) and the pf_cls C ABI.
#include "pf_cls.h"
#include "pf_geom.h"

#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <vector>

namespace pf {
namespace {

constexpr u32 kKeyDropped = 0xFFFFu;
constexpr u32 kKeyGround = 0x8000u;
constexpr size_t kClsCells = (size_t)1 << 23;   // 1 m cells of the U grid

struct ClsDev {          // kernel view of ClsGPU
    pf_cls_params prm;
    int* cnt;
    u32* gb;
    int* gdim;
    u32* cell_cnt;
    u32* cell_minz;
    float* cell_nb;
    u32* pcell;
    u32* keys;
    u32* vals;
    float4* U;
    u32* ckeys;
    u32* cvals;
    uint8_t* code;
    int* ptnum;
    float4* box;
    int* sticky;         // optional: a sticky copy of CC_ERR (the odometry handle's error word)
    u32 cap;             // allocation sizes, for the bounds-checked development build (PF_DEV_BOUNDS)
    u32 cell_cap;
    float4* nrm;         // per U point: the normal assign_normal leaves (pca_code)
};
ClsDev dev_view(ClsGPU& c) {
    return ClsDev{c.prm, c.cnt, c.gb, c.gdim, c.cell_cnt, c.cell_minz, c.cell_nb, c.pcell, c.keys, c.vals,
                  c.U, c.ckeys, c.cvals, c.code, c.ptnum, c.box, c.sticky, (u32)c.cap, (u32)c.grid.cell_cap, c.nrm};
}

// Development build with -DPF_DEV_BOUNDS (tools/build_variant.sh): every indexed global access of the
// front-end kernels is checked against its allocation; a violation sets cnt[CC_ERR] = 2 and, inside
// a BPF handle, its sticky error word (the C ABI then returns PF_ECAPACITY, so a test fails loudly)
// and the access is redirected to element 0. The
// shipped build compiles the checks out. Used to audit the index math (front-end faults).
#ifdef PF_DEV_BOUNDS
#define PF_IDX(d, i, bound) pf_idx_checked((d), (long long)(i), (long long)(bound))
__device__ __forceinline__ long long pf_idx_checked(const ClsDev& d, long long i, long long bound) {
    if (i < 0 || i >= bound) {
        d.cnt[CC_ERR] = 2;
        if (d.sticky) *d.sticky = 2;     // the odometry handle's error word: PF_ECAPACITY at its sync
        return 0;
    }
    return i;
}
#else
#define PF_IDX(d, i, bound) (i)
#endif

__device__ __forceinline__ float wave_minf(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// ---- ground_seg ------------------------------------------------------------------------------

// get_cloud_bbx (:522-556) over x and y; the last workgroup derives row / col / num_grid (:412-415),
// clears the grid (:420-424: min_z = FLT_MAX) and the frame's counters
__global__ void __launch_bounds__(256) k_gs_bounds(const float4* __restrict__ pts, const int* __restrict__ d_n,
                                                   ClsDev d) {
    __shared__ float red[4][4];
    __shared__ int last;
    __shared__ int sdim[3];
    const int n = *d_n;
    float v[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        v[0] = fminf(v[0], p.x); v[1] = fminf(v[1], p.y);
        v[2] = fmaxf(v[2], p.x); v[3] = fmaxf(v[3], p.y);
    }
    const int w = threadIdx.x >> 6;
    v[0] = wave_minf(v[0]); v[1] = wave_minf(v[1]); v[2] = wave_maxf(v[2]); v[3] = wave_maxf(v[3]);
    if (lane_id() == 0)
        for (int k = 0; k < 4; ++k) red[w][k] = v[k];
    __syncthreads();
    if (threadIdx.x < 4) {
        const int k = threadIdx.x;
        float r = red[0][k];
        for (int ww = 1; ww < 4; ++ww) r = k < 2 ? fminf(r, red[ww][k]) : fmaxf(r, red[ww][k]);
        if (k < 2) atomicMin(&d.gb[k], f2ord(r));
        else atomicMax(&d.gb[k], f2ord(r));
    }
    if (threadIdx.x < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(&d.gb[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    if (threadIdx.x == 0) {
        float b[4];
        for (int k = 0; k < 4; ++k) {
            b[k] = ord2f(__hip_atomic_load(&d.gb[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            __hip_atomic_store(&d.gb[k], k < 2 ? 0xFFFFFFFFu : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __hip_atomic_store(&d.gb[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double res = (double)d.prm.gf_grid_res;
        int row = 0, col = 0;
        long long num = 0;
        if (n > 0) {
            row = (int)ceil(((double)b[3] - (double)b[1]) / res);
            col = (int)ceil(((double)b[2] - (double)b[0]) / res);
            num = (long long)row * col;
        }
        int err = 0;
        if (num > kGsMaxCells || num < 0) { num = 0; err = 1; }
        d.gdim[0] = row; d.gdim[1] = col; d.gdim[2] = (int)num;
        d.gdim[4] = __float_as_int(b[0]); d.gdim[5] = __float_as_int(b[1]);
        sdim[0] = (int)num;
        d.cnt[CC_N] = n;
        d.cnt[CC_NU] = 0; d.cnt[CC_NG] = 0;
        for (int k = 0; k < 4; ++k) d.cnt[CC_CLS + k] = 0;
        d.cnt[CC_ERR] = err;
        if (err && d.sticky) *d.sticky = 1;
    }
    __syncthreads();
    const u32 fmax_ord = f2ord(FLT_MAX);
    for (int m = threadIdx.x; m < sdim[0]; m += blockDim.x) {
        d.cell_cnt[m] = 0;
        d.cell_minz[m] = fmax_ord;
    }
}

// :427-448: cell of every point, the cell's point count, its lowest z in (min, max ground height].
// Scan order puts runs of consecutive points into one 3 m cell: a wave takes one count atomic and
// one min atomic per run (up to 16 runs, the rest per lane) instead of serialising on the cell.
__global__ void __launch_bounds__(256) k_gs_assign(const float4* __restrict__ pts, const int* __restrict__ d_n, ClsDev d) {
    const int n = *d_n;
    const int col = d.gdim[1], num = d.gdim[2];
    const double minx = (double)__int_as_float(d.gdim[4]), miny = (double)__int_as_float(d.gdim[5]);
    const double res = (double)d.prm.gf_grid_res;
    const int stride = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i - lane_id() < n; i += stride) {   // wave-uniform
        u32 cell = ~0u;
        float zq = INFINITY;                       // z if it may be the cell's min_z
        if (i < n) {
            const float4 p = pts[i];
            const int tc = (int)floor(((double)p.x - minx) / res);
            const int tr = (int)floor(((double)p.y - miny) / res);
            const long long id = (long long)tr * col + tc;
            if (id >= 0 && id < num) {
                cell = (u32)id;
                if (!(p.z > d.prm.gf_max_ground_height) && p.z > d.prm.gf_min_ground_height && p.z < FLT_MAX)
                    zq = p.z;
            }
            d.pcell[i] = cell;
        }
        u64 todo = __ballot(cell != ~0u);
        for (int it = 0; it < 16 && todo; ++it) {
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const u32 c = (u32)__shfl((int)cell, leader, 64);
            const u64 m = __ballot(cell == c) & todo;
            const float zm = wave_minf(((m >> lane_id()) & 1ull) ? zq : INFINITY);
            if (lane_id() == leader) {
                atomicAdd(&d.cell_cnt[c], (u32)__popcll(m));
                if (zm < INFINITY) atomicMin(&d.cell_minz[c], f2ord(zm));
            }
            todo &= ~m;
        }
        if ((todo >> lane_id()) & 1ull) {
            atomicAdd(&d.cell_cnt[cell], 1u);
            if (zq < INFINITY) atomicMin(&d.cell_minz[cell], f2ord(zq));
        }
    }
}

// :451-467: the 3x3 minimum of min_z for cells off the grid border
__global__ void __launch_bounds__(256) k_gs_nbmin(ClsDev d) {
    const int row = d.gdim[0], col = d.gdim[1], num = d.gdim[2];
    for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < num; m += gridDim.x * blockDim.x) {
        float nb = ord2f(d.cell_minz[m]);
        const int r = m / col, c = m % col;
        if (r >= 1 && r <= row - 2 && c >= 1 && c <= col - 2)
            for (int j = -1; j <= 1; ++j)
                for (int k = -1; k <= 1; ++k) {
                    const float z = ord2f(d.cell_minz[PF_IDX(d, m + j * col + k, num)]);
                    if (nb > z) nb = z;
                }
        d.cell_nb[m] = nb;
    }
}

// :427-494 as a stable sort key: the reference pushes points above the max ground height to
// cloud_unground in input order during the assignment pass, then walks the cells in order pushing
// each cell's remaining points (input order) to ground or non-ground; cells with fewer than
// gf_min_grid_pts points push nothing
// the sorts' digit histograms are fused into their key producers (k_gs_keys, k_u_keys, k_cls_decide:
// sort_hist_*, pf_prims.h), so no separate histogram launch precedes a sort
__global__ void __launch_bounds__(256) k_gs_keys(const float4* __restrict__ pts, const int* __restrict__ d_n, ClsDev d,
                                                  SortHist sh) {
    __shared__ int red[2];
    __shared__ u32 lh[4][256];
    if (threadIdx.x < 2) red[threadIdx.x] = 0;
    sort_hist_begin(lh);
    const int n = *d_n;
    const pf_cls_params& P = d.prm;
    int nu = 0, ng = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32 cell = d.pcell[i];
        const float z = pts[i].z;
#ifdef PF_DEV_BOUNDS
        if (cell != ~0u) (void)PF_IDX(d, cell, d.gdim[2]);
#endif
        u32 key = kKeyDropped;
        if (cell != ~0u) {
            if (z > P.gf_max_ground_height) {
                key = 0;
            } else if ((int)d.cell_cnt[cell] >= P.gf_min_grid_pts) {
                const float minz = ord2f(d.cell_minz[cell]);
                key = 1 + cell;
                if (minz - d.cell_nb[cell] < P.gf_neighbor_height_diff && z - minz < P.gf_max_height_diff &&
                    z > P.gf_min_ground_height)
                    key = kKeyGround + cell;
            }
        }
        nu += key < kKeyGround;
        ng += key >= kKeyGround && key < kKeyDropped;
        d.keys[i] = key;
        d.vals[i] = (u32)i;
        sort_hist_add(lh, key, sh.passes);
    }
    nu = wave_sum_i(nu);
    ng = wave_sum_i(ng);
    if (lane_id() == 0) {
        atomicAdd(&red[0], nu);
        atomicAdd(&red[1], ng);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (red[0]) atomicAdd(&d.cnt[CC_NU], red[0]);
        if (red[1]) atomicAdd(&d.cnt[CC_NG], red[1]);
    }
    sort_hist_end(lh, sh, n, n);
}

// pc2pc (:633-644): the non-ground cloud U in push order, xyz only
__global__ void __launch_bounds__(256) k_gs_gather(const float4* __restrict__ pts, ClsDev d) {
    const int nu = d.cnt[CC_NU];
    if (blockIdx.x == 0 && threadIdx.x == 0) d.cnt[CC_NUG] = nu;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nu; j += gridDim.x * blockDim.x) {
        const float4 p = pts[PF_IDX(d, d.vals[j], d.cnt[CC_N])];
        d.U[j] = make_float4(p.x, p.y, p.z, 0.0f);
    }
}

// groundfilter off: U is the input cloud itself
__global__ void __launch_bounds__(256) k_cls_identity(const float4* __restrict__ pts, const int* __restrict__ d_n, ClsDev d) {
    const int n = *d_n;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        d.cnt[CC_N] = n; d.cnt[CC_NU] = n; d.cnt[CC_NUG] = n; d.cnt[CC_NG] = 0; d.cnt[CC_ERR] = 0;
        for (int k = 0; k < 4; ++k) d.cnt[CC_CLS + k] = 0;
    }
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const float4 p = pts[j];
        d.U[j] = make_float4(p.x, p.y, p.z, 0.0f);
        d.vals[j] = (u32)j;
    }
}

// ---- curvedfilter: DCVC's output becomes the cloud featureExtract sees (src/additionNode.cpp:29-39) --
// the kept points (DCVC's published order) and their input indices into staging, then back over U /
// vals[0 ..) (the ground indices after ground_seg's non-ground count stay where pf_cls_extract reads them)
__global__ void __launch_bounds__(256) k_dc_gather(ClsDev d, const u32* __restrict__ idx, const int* __restrict__ ddim,
                                                    float4* __restrict__ tu, u32* __restrict__ tv) {
    const int nk = ddim[D_NKEPT];
    if (blockIdx.x == 0 && threadIdx.x == 0 && ddim[D_ERR]) {       // too many rings / clusters
        d.cnt[CC_ERR] = 3;
        if (d.sticky) *d.sticky = 3;
    }
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nk; j += gridDim.x * blockDim.x) {
        const u32 u = idx[j];
        tu[j] = d.U[u];
        tv[j] = d.vals[u];
    }
}
__global__ void __launch_bounds__(256) k_dc_commit(ClsDev d, const int* __restrict__ ddim, const float4* __restrict__ tu,
                                                    const u32* __restrict__ tv) {
    const int nk = ddim[D_ERR] ? 0 : ddim[D_NKEPT];
    if (blockIdx.x == 0 && threadIdx.x == 0) d.cnt[CC_NU] = nk;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nk; j += gridDim.x * blockDim.x) {
        d.U[j] = tu[j];
        d.vals[j] = tv[j];
    }
}

// ---- featureExtract ----------------------------------------------------------------------------

// The U grid: 1 m cells (pf_knn.h) whose points are ordered inside each cell by the Morton code of
// their 0.125 m sub-cell, so that every aligned 16-point chunk of the cell-ordered array is compact;
// the chunks' bounding boxes let the search skip chunks the way a kd-tree skips leaves.
__device__ __forceinline__ u32 morton3(u32 x, u32 y, u32 z) {
    u32 m = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) m |= (((x >> b) & 1u) << (3 * b)) | (((y >> b) & 1u) << (3 * b + 1)) | (((z >> b) & 1u) << (3 * b + 2));
    return m;
}
__device__ __forceinline__ u32 sub8(float v) {
    const float f = (v - floorf(v)) * 8.0f;
    const int s = (int)f;
    return (u32)(s < 0 ? 0 : (s > 7 ? 7 : s));
}
__global__ void __launch_bounds__(256) k_u_keys(ClsDev d, const int* __restrict__ dm, SortHist sh) {
    __shared__ u32 lh[4][256];
    sort_hist_begin(lh);
    const int nu = d.cnt[CC_NU];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nu; j += gridDim.x * blockDim.x) {
        const float4 p = d.U[j];
        u32 key = 0;
        if (dm[7]) {
            const int x = (int)floorf(p.x) - dm[0], y = (int)floorf(p.y) - dm[1], z = (int)floorf(p.z) - dm[2];
            const u32 cell = (u32)PF_IDX(d, (long long)dm[6] + (long long)(z * dm[4] + y) * dm[3] + x, d.cell_cap);
            key = (cell << 9) | morton3(sub8(p.x), sub8(p.y), sub8(p.z));
        }
        d.ckeys[j] = key;
        d.cvals[j] = (u32)j;
        sort_hist_add(lh, key, sh.passes);
    }
    sort_hist_end(lh, sh, nu, nu);
}
// cell-ordered points (w = U index), and the counts left zero for the next build
__global__ void __launch_bounds__(256) k_u_place(ClsDev d, float4* __restrict__ cpts, u32* __restrict__ cell_count,
                                                 const int* __restrict__ dm, u32* __restrict__ ttot, int ttiles) {
    const int nu = d.cnt[CC_NU];
    if (blockIdx.x == 0)                          // the grid scan's tile totals, for the next build
        for (int j = threadIdx.x; j < ttiles; j += blockDim.x) ttot[j] = 0u;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nu; i += gridDim.x * blockDim.x) {
        const u32 j = d.cvals[i];
        const float4 p = d.U[PF_IDX(d, j, nu)];
        cpts[i] = make_float4(p.x, p.y, p.z, __int_as_float((int)j));
        if (dm[7]) cell_count[d.ckeys[i] >> 9] = 0u;
    }
}
// bounding box of every aligned 16-point chunk (a DPP row per chunk)
__global__ void __launch_bounds__(256) k_u_boxes(ClsDev d, const float4* __restrict__ cpts) {
    const int nu = d.cnt[CC_NU];
    const int nch = (nu + 15) / 16;
    const int l = threadIdx.x & 15;
    for (int c = (blockIdx.x * blockDim.x + threadIdx.x) / 16; c - (int)(threadIdx.x & 63) / 16 < nch;
         c += gridDim.x * blockDim.x / 16) {
        const int i = c * 16 + l;
        float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
        if (c < nch && i < nu) {
            const float4 p = cpts[i];
            lo = make_float4(p.x, p.y, p.z, 0.f);
            hi = lo;
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            lo.x = fminf(lo.x, __shfl_xor(lo.x, o, 64)); lo.y = fminf(lo.y, __shfl_xor(lo.y, o, 64));
            lo.z = fminf(lo.z, __shfl_xor(lo.z, o, 64));
            hi.x = fmaxf(hi.x, __shfl_xor(hi.x, o, 64)); hi.y = fmaxf(hi.y, __shfl_xor(hi.y, o, 64));
            hi.z = fmaxf(hi.z, __shfl_xor(hi.z, o, 64));
        }
        if (c < nch && l == 0) {
            d.box[2 * c] = lo;
            d.box[2 * c + 1] = hi;
        }
    }
}

// PCA of the neighbourhood nb[0 .. n) (ascending distance) and the class decision, :653-688 /
// :283-323, f32 as pcl::PCA computes it; the eigen-decomposition is the f64 cyclic Jacobi (eig3)
// of the f32 covariance, rounded back to f32. Returns the index_with_feature code; nrm receives what
// assign_normal (:327-346) leaves in the point: get_pc_pca_feature writes (normal direction,
// planar_2) into every point with more than 3 neighbours (:238-239; with 2-3 the zero-initialised
// feature, :206), featureExtract then overwrites pillar and beam points with (principal direction,
// linear_2) (:663-674); zeros for 0-3 neighbours.
template <class Get>
__device__ int pca_code(Get get, int n, float qz, const pf_cls_params& P, float4& nrm) {
    nrm = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n <= 3) return 0;
#ifdef PF_DEV_NOPCA
    return 3;                                  // development: the search without the PCA (timing only)
#endif
    float sx = 0.f, sy = 0.f, sz = 0.f;
    for (int e = 0; e < n; ++e) {
        const float4 p = get(e);
        sx += p.x; sy += p.y; sz += p.z;
    }
    const float fn = (float)n;
    const float mx = sx / fn, my = sy / fn, mz = sz / fn;
    float cxx = 0.f, cxy = 0.f, cxz = 0.f, cyy = 0.f, cyz = 0.f, czz = 0.f;
    for (int e = 0; e < n; ++e) {              // the neighbours again (L2-resident) instead of a copy
        const float4 p = get(e);
        const float dx = p.x - mx, dy = p.y - my, dz = p.z - mz;
        cxx += dx * dx; cxy += dx * dy; cxz += dx * dz;
        cyy += dy * dy; cyz += dy * dz; czz += dz * dz;
    }
    double A[3][3] = {{cxx, cxy, cxz}, {cxy, cyy, cyz}, {cxz, cyz, czz}};
    double ev[3], V[3][3];
    eig3(A, ev, V);
    const float l1 = (float)ev[2], l2 = (float)ev[1], l3 = (float)ev[0];
    float v0[3] = {(float)V[0][2], (float)V[1][2], (float)V[2][2]};
    const float v1[3] = {(float)V[0][1], (float)V[1][1], (float)V[2][1]};
    float nv[3] = {v0[1] * v1[2] - v0[2] * v1[1], v0[2] * v1[0] - v0[0] * v1[2], v0[0] * v1[1] - v0[1] * v1[0]};
    float sq = v0[0] * v0[0] + v0[1] * v0[1] + v0[2] * v0[2];
    if (sq > 0.f) { const float s = sqrtf(sq); v0[0] /= s; v0[1] /= s; v0[2] /= s; }
    sq = nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2];
    if (sq > 0.f) { const float s = sqrtf(sq); nv[0] /= s; nv[1] /= s; nv[2] /= s; }
    const double d1 = l1, d2 = l2, d3 = l3;
    const double linear_2 = (d1 - d2) / d1;
    const double planar_2 = (d2 - d3) / d1;
    nrm = make_float4(nv[0], nv[1], nv[2], (float)planar_2);    // assign_normal(plane), :238-239
    if (!(n > P.k_min)) return 0;                               // :657
    if (linear_2 > (double)P.edge_thre) {
        const float4 pr = make_float4(v0[0], v0[1], v0[2], (float)linear_2);
        if (fabsf(v0[2]) > P.linear_vsin_high) { nrm = pr; return 1; }
        if (fabsf(v0[2]) < P.linear_vsin_low && qz < P.beam_h_max && qz > P.beam_h_min) { nrm = pr; return 2; }
    } else if (planar_2 > (double)P.planar_thre) {
        if (fabsf(nv[2]) < P.planar_vsin_low) return 3;
    }
    return 0;
}

__device__ __forceinline__ u64 shfl_u64(u64 v, int src) {
    const int lo = __shfl((int)(u32)v, src, 64), hi = __shfl((int)(u32)(v >> 32), src, 64);
    return ((u64)(u32)hi << 32) | (u64)(u32)lo;
}
__device__ __forceinline__ u64 shfl_xor_u64(u64 v, int m) {
    const int lo = __shfl_xor((int)(u32)v, m, 64), hi = __shfl_xor((int)(u32)(v >> 32), m, 64);
    return ((u64)(u32)hi << 32) | (u64)(u32)lo;
}
#ifndef PF_CLS_BATCH
#define PF_CLS_BATCH 16
#endif
#ifndef PF_CLS_NOSORT
#define PF_CLS_NOSORT 0
#endif
constexpr int kClsNoSort = PF_CLS_NOSORT;   // open chunks in a round up to which the round is not sorted (0: a round
                                            // without open chunks skips its sort; 4 measured 249 vs 244 us)
#ifdef PF_CLS_ROWS_PLAIN
__constant__ constexpr int kClsRowOrder[9] = {0, 1, 2, 3, 4, 5, 6, 7, 8};
#else
__constant__ constexpr int kClsRowOrder[9] = {4, 1, 3, 5, 7, 0, 2, 6, 8};   // row r = (oz + 1) * 3 + oy + 1
#endif
#ifndef PF_CLS_MINX
#define PF_CLS_MINX 0   // 1: passes take their chunks by wave minima, no round sort (266.6 vs 238.3 us, off)
#endif
#ifndef PF_CLS_PHASES
#define PF_CLS_PHASES 1
#endif
// 2: the query's own row first, then the other eight re-cut by the k-th distance (fewer rounds and
// chunks, but 281 vs 238 us in one A/B run: the phase loop costs more than the rounds it saves)
constexpr int kClsPhases = PF_CLS_PHASES;
constexpr int kBatch = PF_CLS_BATCH;   // winners in one pass above which the pass is merged as a whole
__device__ __forceinline__ u64 readlane_u64(u64 v, int lane) {
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)v, lane);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), lane);
    return ((u64)hi << 32) | (u64)lo;
}
// lane l takes lane l - 1's value, lane 0 takes 0 (DPP wave_shr:1)
__device__ __forceinline__ u64 wave_shr1_u64(u64 v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(u32)v, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(u32)(v >> 32), 0x138, 0xf, 0xf, true);
    return ((u64)(u32)hi << 32) | (u64)(u32)lo;
}

// ascending sort of one u64 per lane across the wave (bitonic network)
__device__ __forceinline__ u64 wave_sort_u64(u64 v) {
    const int l = lane_id();
#pragma unroll
    for (int kk = 2; kk <= 64; kk <<= 1)
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            const u64 o = shfl_xor_u64(v, j);
            v = (((l & j) == 0) == ((l & kk) == 0)) ? (o < v ? o : v) : (o > v ? o : v);
        }
    return v;
}

__device__ __forceinline__ u32 wave_sort_u32(u32 v) {
    const int l = lane_id();
#pragma unroll
    for (int kk = 2; kk <= 64; kk <<= 1)
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            const u32 o = (u32)__shfl_xor((int)v, j, 64);
            v = (((l & j) == 0) == ((l & kk) == 0)) ? (o < v ? o : v) : (o > v ? o : v);
        }
    return v;
}

#ifdef PF_DEV_CLS_STATS
// development (tools/build_variant.sh NAME -DPF_DEV_CLS_STATS): per-query work counters of the search,
// summed over a call and printed by k_cls_decide's first thread: queries, chunk rounds, chunks in the
// rows, chunks opened, read passes, candidates in range, candidates inside r, batch merges, single inserts
__device__ unsigned long long g_cls_stats[10];
#define CLS_STAT(i, v) do { if (lane_id() == 0) atomicAdd(&g_cls_stats[i], (unsigned long long)(v)); } while (0)
#else
#define CLS_STAT(i, v) do { } while (0)
#endif
// KdTreeFLANN::radiusSearch(i, r, idx, d2, k) for every U point, one wave per query. The candidates
// are the 27 cells of the 1 m grid around the query (every point with d^2 < r^2 <= 1 lies there,
// pf_knn.h), i.e. the aligned 16-point chunks of the cell-ordered cloud that overlap the 9 x-rows.
// Per round of 64 chunks, every lane bounds one chunk (its box's float lower bound of d^2, exact by
// the monotone-rounding argument of pf_knn.h) and the wave sorts the (bound, chunk) pairs; chunks are
// then read nearest first, 4 per pass (16 lanes each), and the round ends at the first bound above
// the k-th distance. The sorted list of the k best keys (d^2 bits, index) lives in registers, entry j
// on lane j: the first pass and any pass with more than kBatch winners merge by a bitonic network,
// single winners by one wave shift (keys are distinct). Writes the neighbour lists and sizes.
__global__ void __launch_bounds__(256) k_cls_search(ClsDev d, GridView gv, u32* __restrict__ nbr) {
    constexpr int WPB = 4;
    const int K = d.prm.k;
    const float r2 = (float)((double)d.prm.radius * (double)d.prm.radius);
    const int nu = d.cnt[CC_NU];
    const int* dm = gv.dims;
    const int l = lane_id();
    const int nw = gridDim.x * WPB;
    const int wv = (int)xcd_block(blockIdx.x, gridDim.x) * WPB + (int)(threadIdx.x >> 6);
    for (int qs = wv; qs < nu; qs += nw) {                   // wave-uniform
        // queries in cell (Morton) order: neighbouring waves share candidate chunks in L2
        const float4 qc = gv.cpts[PF_IDX(d, qs, d.cap)];
        const int q = __float_as_int(qc.w);
        const float4 qp = make_float4(qc.x, qc.y, qc.z, 0.f);
        u64 ent = ~0ull;                                     // list entry l
        u64 thr = ~0ull;                                     // entry K - 1
        auto open = [&](float lb) {
            return lb < r2 && (thr == ~0ull || lb <= __uint_as_float((u32)(thr >> 32)));
        };
        auto box_lb = [&](int c) {
            const float4 lo = d.box[PF_IDX(d, 2 * c, 2 * (d.cap / 16 + 1))];
            const float4 hi = d.box[PF_IDX(d, 2 * c + 1, 2 * (d.cap / 16 + 1))];
            const float tx = qp.x < lo.x ? lo.x - qp.x : (qp.x > hi.x ? qp.x - hi.x : 0.0f);
            const float ty = qp.y < lo.y ? lo.y - qp.y : (qp.y > hi.y ? qp.y - hi.y : 0.0f);
            const float tz = qp.z < lo.z ? lo.z - qp.z : (qp.z > hi.z ? qp.z - hi.z : 0.0f);
            return (0.0f + tx * tx + ty * ty) + tz * tz;
        };
        auto merge_batch = [&](u64 key) {                    // all keys of a pass below thr, at once
            u64 v = wave_sort_u64(key < thr ? key : ~0ull);
            if (readlane_u64(ent, 0) == ~0ull) {             // empty list: the sorted batch's 32 smallest
                ent = l < 32 ? v : ~0ull;
                thr = readlane_u64(ent, K - 1);
                return;
            }
            const u64 rev = shfl_u64(v, 63 - l);             // lanes 32.. : the 32 smallest, descending
            v = l < 32 ? ent : rev;                          // bitonic: list ascending, keys descending
#pragma unroll
            for (int j = 32; j > 0; j >>= 1) {
                const u64 o = shfl_xor_u64(v, j);
                v = (l & j) == 0 ? (o < v ? o : v) : (o > v ? o : v);
            }
            ent = v;
            thr = readlane_u64(ent, K - 1);
        };
        if (dm[7]) {
            const float fcx = floorf(qp.x), fcy = floorf(qp.y), fcz = floorf(qp.z);
            const int cx = (int)fcx, cy = (int)fcy, cz = (int)fcz;
            const int minx = dm[0], miny = dm[1], minz = dm[2], dx = dm[3], dy = dm[4], dz = dm[5], base = dm[6];
            const float lx = qp.x - fcx, hx = (fcx + 1.0f) - qp.x;
            const float ly = qp.y - fcy, hy = (fcy + 1.0f) - qp.y;
            const float lz = qp.z - fcz, hz = (fcz + 1.0f) - qp.z;
            const int xi = cx - minx;                          // the query's own cell is in the grid
            // lane r < 9 loads x-row r's cell boundaries (r = (oz + 1) * 3 + oy + 1): starts of cells
            // xi - 1, xi, xi + 1 and the end of xi + 1
            u32 w0 = 0, w1 = 0, w2 = 0, w3 = 0;
            if (l < 9) {
                const int y = cy + l % 3 - 1 - miny, z = cz + l / 3 - 1 - minz;
                if (y >= 0 && y < dy && z >= 0 && z < dz) {
                    const long long c0 = (long long)base + (long long)(z * dy + y) * dx + xi;
                    const u32* cs = gv.cell_start;
                    w1 = cs[PF_IDX(d, c0, d.cell_cap + 1)];
                    w2 = cs[PF_IDX(d, c0 + 1, d.cell_cap + 1)];
                    w0 = xi > 0 ? cs[PF_IDX(d, c0 - 1, d.cell_cap + 1)] : w1;
                    w3 = xi + 1 < dx ? cs[PF_IDX(d, c0 + 2, d.cell_cap + 1)] : w2;
                }
            }
            // Two phases: the query's own row, then the other eight with their ranges cut by the k-th
            // distance found in the first (with a full list most of them close at once). Per phase:
            // each row's point range [ra, rb) (end cells dropped when their bound cannot hold a
            // winner: >= r^2, or above the k-th distance) and the prefix of the rows' chunk counts
            bool first = true;
            CLS_STAT(0, 1);
            for (int ph = 0; ph < kClsPhases; ++ph) {
            u32 ra[9], rb[9], pre[9];
            u32 total = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                // rows in processing order: the query's own row, the four sharing a face with it,
                // then the four diagonal ones (the nearest candidates fill the list first)
                const int r = kClsRowOrder[k];
                const int oy = r % 3 - 1, oz = r / 3 - 1;
                const u32 s0 = (u32)__builtin_amdgcn_readlane((int)w0, r), s1 = (u32)__builtin_amdgcn_readlane((int)w1, r);
                const u32 s2 = (u32)__builtin_amdgcn_readlane((int)w2, r), s3 = (u32)__builtin_amdgcn_readlane((int)w3, r);
                const float by = oy < 0 ? ly : (oy > 0 ? hy : 0.0f);
                const float bz = oz < 0 ? lz : (oz > 0 ? hz : 0.0f);
                const float brow = (0.0f + by * by) + bz * bz;
                const float bl = (lx * lx + by * by) + bz * bz;
                const float bh = (hx * hx + by * by) + bz * bz;
                u32 a0 = open(bl) ? s0 : s1, b0 = open(bh) ? s3 : s2;
                const bool in_phase = kClsPhases == 1 || (ph == 0 ? k == 0 : k > 0);
                if (!in_phase || !open(brow) || a0 >= b0) a0 = b0 = 0;
                ra[k] = a0;
                rb[k] = b0;
                pre[k] = total;
                total += a0 < b0 ? ((b0 - 1) >> 4) - (a0 >> 4) + 1 : 0;
            }
            // chunk ordinal t -> (chunk, its row's range)
            auto locate = [&](u32 t, u32& chunk, u32& a0, u32& b0) {
                int k = 0;
#pragma unroll
                for (int r = 1; r < 9; ++r) k = t >= pre[r] ? r : k;
                u32 pk = pre[0], ak = ra[0], bk = rb[0];
#pragma unroll
                for (int r = 1; r < 9; ++r) {
                    pk = k == r ? pre[r] : pk;
                    ak = k == r ? ra[r] : ak;
                    bk = k == r ? rb[r] : bk;
                }
                chunk = (ak >> 4) + (t - pk);
                a0 = ak;
                b0 = bk;
            };
            // sort keys: the bound's float bits with the low 6 bits replaced by the chunk's lane in the
            // round (truncation only lowers a bound, so stopping at the first truncated bound above
            // the k-th distance stays exact; a chunk is still read only if its bound may hold a winner)
            CLS_STAT(2, total);
            for (u32 g = 0; g < total; g += 64) {
                CLS_STAT(1, 1);
                const u32 t = g + (u32)l;
                u32 sk = ~0u;
                if (t < total) {
                    u32 c, a0, b0;
                    locate(t, c, a0, b0);
                    const float lb = box_lb((int)c);
                    if (open(lb)) sk = (__float_as_uint(lb) & ~0x3Fu) | (u32)l;
                }
                u64 om = __ballot(sk != ~0u);
                const int nopen = __popcll(om);
                CLS_STAT(3, nopen);
#if PF_CLS_MINX
                // nearest first without the sort: each pass takes the four smallest open bounds by
                // wave minima (a key's low 6 bits are its lane, so the minimum names its lane)
                u32 rem = sk;
                auto take_min = [&]() {
                    u32 m = rem;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const u32 v = (u32)__shfl_xor((int)m, o, 64);
                        m = v < m ? v : m;
                    }
                    m = (u32)__builtin_amdgcn_readfirstlane((int)m);
                    if (m != ~0u && l == (int)(m & 0x3Fu)) rem = ~0u;
                    return m;
                };
                if (!om) continue;
                const bool few = false;
                u32 f0 = ~0u, f1 = ~0u, f2 = ~0u, f3 = ~0u;
                (void)f0; (void)f1; (void)f2; (void)f3;
#else
                // up to one pass of open chunks: read them as they lie (no sort); else nearest first
                const bool few = nopen <= kClsNoSort;
                u32 f0 = ~0u, f1 = ~0u, f2 = ~0u, f3 = ~0u;
                if (few) {
                    if (!om) continue;
                    f0 = (u32)__builtin_amdgcn_readlane((int)sk, __ffsll((unsigned long long)om) - 1);
                    om &= om - 1;
                    if (om) f1 = (u32)__builtin_amdgcn_readlane((int)sk, __ffsll((unsigned long long)om) - 1);
                    if (om) om &= om - 1;
                    if (om) f2 = (u32)__builtin_amdgcn_readlane((int)sk, __ffsll((unsigned long long)om) - 1);
                    if (om) om &= om - 1;
                    if (om) f3 = (u32)__builtin_amdgcn_readlane((int)sk, __ffsll((unsigned long long)om) - 1);
                } else {
                    sk = wave_sort_u32(sk);
                }
#endif
                auto lb_of = [](u32 k) { return __uint_as_float(k & ~0x3Fu); };
                for (int i = 0; i < nopen; i += 4) {
#if PF_CLS_MINX
                    const u32 k0 = take_min();
                    if (!open(lb_of(k0))) break;                   // ascending: the rest are closed too
                    const u32 k1 = i + 1 < nopen ? take_min() : ~0u;
                    const u32 k2 = i + 2 < nopen ? take_min() : ~0u;
                    const u32 k3 = i + 3 < nopen ? take_min() : ~0u;
                    const int j = i + (l >> 4);
                    CLS_STAT(4, 1);
#else
                    // sorted: a closed chunk closes the rest too
                    if (!few && !open(lb_of((u32)__builtin_amdgcn_readlane((int)sk, i)))) break;
                    const int j = i + (l >> 4);
                    CLS_STAT(4, 1);
                    const u32 k0 = few ? f0 : (u32)__builtin_amdgcn_readlane((int)sk, i);
                    const u32 k1 = few ? f1 : (u32)__builtin_amdgcn_readlane((int)sk, i + 1 < 64 ? i + 1 : 63);
                    const u32 k2 = few ? f2 : (u32)__builtin_amdgcn_readlane((int)sk, i + 2 < 64 ? i + 2 : 63);
                    const u32 k3 = few ? f3 : (u32)__builtin_amdgcn_readlane((int)sk, i + 3 < 64 ? i + 3 : 63);
#endif
                    const u32 sj = (l >> 4) == 1 ? k1 : ((l >> 4) == 2 ? k2 : ((l >> 4) == 3 ? k3 : k0));
                    u64 key = ~0ull;
                    if (j < nopen && open(lb_of(sj))) {
                        u32 c, a0, b0;
                        locate(g + (sj & 0x3Fu), c, a0, b0);
                        const u32 v = c * 16u + (u32)(l & 15);
                        if (v >= a0 && v < b0) {
#ifdef PF_DEV_CLS_STATS
                            atomicAdd(&g_cls_stats[5], 1ull);
#endif
                            const float4 p = gv.cpts[PF_IDX(d, v, nu)];
                            const float dd = knn_d2(qp.x, qp.y, qp.z, p);
                            if (dd < r2) key = knn_key(dd, __float_as_int(p.w));
                        }
                    }
                    u64 sm = __ballot(key < thr);
#ifdef PF_DEV_CLS_STATS
                    {
                        const u64 inr = __ballot(key != ~0ull);
                        CLS_STAT(6, __popcll(inr));
                    }
#endif
                    if (first || __popcll(sm) > kBatch) {
                        if (sm) CLS_STAT(7, 1);
                        if (sm) merge_batch(key);
                        first = false;
                        continue;
                    }
                    while (sm) {
                        const int sl = __ffsll((unsigned long long)sm) - 1;
                        sm &= sm - 1;
                        const u64 kk = readlane_u64(key, sl);
                        if (!(kk < thr)) continue;
                        CLS_STAT(8, 1);
                        const u64 prev = wave_shr1_u64(ent);
                        ent = kk < prev ? prev : (kk < ent ? kk : ent);
                        thr = readlane_u64(ent, K - 1);
                    }
                }
            }
            }
        }
        const int found = __popcll(__ballot(l < K && ent != ~0ull));
        if (l < found) nbr[PF_IDX(d, (size_t)q * kClsMaxK + l, (long long)d.cap * kClsMaxK)] = (u32)(ent & 0xffffffffull);
        if (l == 0) d.ptnum[PF_IDX(d, q, nu)] = found;
    }
}

// PCA + decision, one thread per U point over its neighbour list (ascending distance)
__global__ void __launch_bounds__(256) k_cls_decide(ClsDev d, const u32* __restrict__ nbr, SortHist sh) {
    __shared__ int ccount[4];
    __shared__ u32 lh[4][256];
    if (threadIdx.x < 4) ccount[threadIdx.x] = 0;
    sort_hist_begin(lh);
    const int nu = d.cnt[CC_NU];
#ifdef PF_DEV_CLS_STATS
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        unsigned long long* g = g_cls_stats;
        printf("CLS_STATS q=%llu rounds=%llu chunks=%llu opened=%llu passes=%llu inrange=%llu inr=%llu merges=%llu inserts=%llu\n",
               g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8]);
        for (int i = 0; i < 10; ++i) g[i] = 0ull;
    }
#endif
    int local[4] = {0, 0, 0, 0};
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nu; q += gridDim.x * blockDim.x) {
        const int n = d.ptnum[q];
        const u32* lst = nbr + (size_t)q * kClsMaxK;
        const float4* U = d.U;
#ifdef PF_DEV_BOUNDS
        if (n > d.prm.k) (void)PF_IDX(d, n, 0);             // a list longer than k: flagged
#endif
        float4 nv;
        const int code = pca_code([&](int e) { return U[PF_IDX(d, lst[e], nu)]; }, n, U[q].z, d.prm, nv);
        d.nrm[q] = nv;
        const u32 key = code == 2 ? 0u : (code == 1 ? 1u : (code == 3 ? 2u : 3u));   // beam, pillar, facade, none
        d.code[q] = (uint8_t)code;
        d.ckeys[q] = key;
        d.cvals[q] = (u32)q;
        local[key]++;
        sort_hist_add(lh, key, sh.passes);
    }
    for (int k = 0; k < 4; ++k) {
        const int v = wave_sum_i(local[k]);
        if (lane_id() == 0 && v) atomicAdd(&ccount[k], v);
    }
    __syncthreads();
    if (threadIdx.x < 4 && ccount[threadIdx.x]) atomicAdd(&d.cnt[CC_CLS + threadIdx.x], ccount[threadIdx.x]);
    sort_hist_end(lh, sh, nu, nu);
}

// the three clouds (U order within a class) and, optionally, their input indices
__global__ void __launch_bounds__(256) k_cls_out(ClsDev d, const u32* __restrict__ ks, const u32* __restrict__ vs,
                                                 float4* o0, float4* o1, float4* o2, int* c0, int* c1, int* c2,
                                                 int* idx_out) {
    const int nu = d.cnt[CC_NU];
    const int n0 = d.cnt[CC_CLS], n1 = d.cnt[CC_CLS + 1], n2 = d.cnt[CC_CLS + 2];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (c0) *c0 = n0;
        if (c1) *c1 = n1;
        if (c2) *c2 = n2;
    }
    const int nout = n0 + n1 + n2;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nout && j < nu; j += gridDim.x * blockDim.x) {
        const u32 k = ks[j];
        const u32 u = vs[j];
        const int pos = j - (k > 0 ? n0 : 0) - (k > 1 ? n1 : 0);
        float4* o = k == 0 ? o0 : (k == 1 ? o1 : o2);
        if (o) o[PF_IDX(d, pos, nout)] = d.U[PF_IDX(d, u, nu)];
        if (idx_out) idx_out[j] = (int)d.vals[u];
    }
}

constexpr int kEwBlocks = 512;

}  // namespace

int cls_alloc(ClsGPU& c, size_t cap) {
    c.cap = cap;
    const size_t cells = kGsMaxCells;
    if (hipMalloc(&c.cnt, sizeof(int) * CC_COUNT) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.gb, sizeof(u32) * 8) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.gdim, sizeof(int) * 8) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.cell_cnt, sizeof(u32) * cells) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.cell_minz, sizeof(u32) * cells) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.cell_nb, sizeof(float) * cells) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.pcell, sizeof(u32) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.keys, sizeof(u32) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.vals, sizeof(u32) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.pts, sizeof(float4) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.U, sizeof(float4) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.ckeys, sizeof(u32) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.cvals, sizeof(u32) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.code, cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.ptnum, sizeof(int) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.idx_out, sizeof(int) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.nbr, sizeof(u32) * kClsMaxK * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.box, sizeof(float4) * 2 * (cap / 16 + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&c.nrm, sizeof(float4) * cap) != hipSuccess) return PF_ENOMEM;
    const u32 gb0[8] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u, 0u, 0u, 0u};
    if (hipMemcpy(c.gb, gb0, sizeof(gb0), hipMemcpyHostToDevice) != hipSuccess) return PF_EHIP;
    if (hipMemset(c.cnt, 0, sizeof(int) * CC_COUNT) != hipSuccess) return PF_EHIP;
    int rc = grid_alloc(c.grid, cap, kClsCells);
    if (rc) return rc;
    return prim_alloc(c.w, cap, kClsCells + 2);
}

int cls_set_dcvc(ClsGPU& c, const pf_dcvc_params* p) {
    if (!p) {
        if (c.dcvc) {
            dcvc_free(*c.dcvc);
            delete c.dcvc;
            c.dcvc = nullptr;
        }
        return PF_OK;
    }
    if (!dcvc_params_valid(p)) return PF_EINVAL;
    if (!c.dcvc) {
        c.dcvc = new DcvcGPU();
        int rc = dcvc_alloc(*c.dcvc, c.cap);
        if (rc == PF_OK && !c.dU && hipMalloc(&c.dU, sizeof(float4) * c.cap) != hipSuccess) rc = PF_ENOMEM;
        if (rc == PF_OK && !c.dV && hipMalloc(&c.dV, sizeof(u32) * c.cap) != hipSuccess) rc = PF_ENOMEM;
        if (rc) {
            dcvc_free(*c.dcvc);
            delete c.dcvc;
            c.dcvc = nullptr;
            return rc;
        }
    }
    return dcvc_set_params(*c.dcvc, *p);
}

void cls_free(ClsGPU& c) {
    void* ps[] = {c.cnt, c.gb, c.gdim, c.cell_cnt, c.cell_minz, c.cell_nb, c.pcell, c.keys, c.vals, c.pts,
                  c.U, c.ckeys, c.cvals, c.code, c.ptnum, c.idx_out, c.box, c.nbr, c.nrm};
    for (void* p : ps) (void)hipFree(p);
    (void)cls_set_dcvc(c, nullptr);
    (void)hipFree(c.dU);
    (void)hipFree(c.dV);
    grid_free(c.grid);
    prim_free(c.w);
    c = ClsGPU{};
}

void cls_enqueue(ClsGPU& c, const float4* d_pts, const int* d_n, float4* const* out, int* const* out_cnt,
                 bool idx, hipStream_t s, bool ground_only) {
    ClsDev d = dev_view(c);
    if (c.prm.ground_filter) {
        hipLaunchKernelGGL(k_gs_bounds, dim3(64), dim3(256), 0, s, d_pts, d_n, d);
        hipLaunchKernelGGL(k_gs_assign, dim3(kEwBlocks), dim3(256), 0, s, d_pts, d_n, d);
        hipLaunchKernelGGL(k_gs_nbmin, dim3(128), dim3(256), 0, s, d);
        hipLaunchKernelGGL(k_gs_keys, dim3(kEwBlocks), dim3(256), 0, s, d_pts, d_n, d, sort_hist(c.w, 16, true));
        radix_sort_pairs(c.keys, c.vals, d_n, 16, c.w, s, nullptr, nullptr, true);
        hipLaunchKernelGGL(k_gs_gather, dim3(kEwBlocks), dim3(256), 0, s, d_pts, d);
    } else {
        hipLaunchKernelGGL(k_cls_identity, dim3(kEwBlocks), dim3(256), 0, s, d_pts, d_n, d);
    }
    if (ground_only) return;
    if (c.dcvc) {                                    // curvedfilter: DCVC on the non-ground cloud
        u32* kept = nullptr;
        dcvc_enqueue(*c.dcvc, c.U, c.cnt + CC_NU, s, &kept);
        hipLaunchKernelGGL(k_dc_gather, dim3(kEwBlocks), dim3(256), 0, s, d, kept, c.dcvc->dim, c.dU, c.dV);
        hipLaunchKernelGGL(k_dc_commit, dim3(kEwBlocks), dim3(256), 0, s, d, c.dcvc->dim, c.dU, c.dV);
    }
    GridPtrs gp{};
    gp.m[0] = c.U;
    gp.n[0] = c.cnt + CC_NU;
    gp.nm = 1;
    grid_count_scan(c.grid, gp, c.w, s);
    hipLaunchKernelGGL(k_u_keys, dim3(kEwBlocks), dim3(256), 0, s, d, c.grid.dims, sort_hist(c.w, 32, true));
    radix_sort_pairs(c.ckeys, c.cvals, c.cnt + CC_NU, 32, c.w, s, nullptr, nullptr, true);
    hipLaunchKernelGGL(k_u_place, dim3(kEwBlocks), dim3(256), 0, s, d, c.grid.cpts, c.grid.cell_count, c.grid.dims,
                       c.grid.ttot, c.grid.ttiles);
    hipLaunchKernelGGL(k_u_boxes, dim3(kEwBlocks), dim3(256), 0, s, d, c.grid.cpts);
    const GridView gv{c.grid.dims, c.grid.cell_start, c.grid.cpts};
    hipLaunchKernelGGL(k_cls_search, dim3(4096), dim3(256), 0, s, d, gv, c.nbr);
    hipLaunchKernelGGL(k_cls_decide, dim3(kEwBlocks), dim3(256), 0, s, d, c.nbr, sort_hist(c.w, 8, false));
    u32 *ks = nullptr, *vs = nullptr;
    radix_sort_pairs(c.ckeys, c.cvals, c.cnt + CC_NU, 8, c.w, s, &ks, &vs, true);
    hipLaunchKernelGGL(k_cls_out, dim3(kEwBlocks), dim3(256), 0, s, d, ks, vs, out ? out[0] : nullptr,
                       out ? out[1] : nullptr, out ? out[2] : nullptr, out_cnt ? out_cnt[0] : nullptr,
                       out_cnt ? out_cnt[1] : nullptr, out_cnt ? out_cnt[2] : nullptr, idx ? c.idx_out : nullptr);
}

}  // namespace pf

// ==================================================================================================
// pf_cls C ABI
// ==================================================================================================
using namespace pf;

struct pf_cls {
    int device = 0;
    hipStream_t stream = nullptr;
    ClsGPU c;
    int* d_n = nullptr;
    std::vector<float4> host;
};

namespace {
bool cls_params_ok(const pf_cls_params* p) {
    return p && p->k >= 1 && p->k <= kClsMaxK && p->radius > 0.f && p->radius <= 1.0f && p->gf_grid_res > 0.f;
}
void repack_xyz(const float* src, size_t n, size_t stride, std::vector<float4>& out) {
    out.resize(n);
    const char* b = reinterpret_cast<const char*>(src);
    for (size_t i = 0; i < n; ++i) {
        const float* p = reinterpret_cast<const float*>(b + i * stride);
        out[i] = make_float4(p[0], p[1], p[2], 0.f);
    }
}
int cls_run(pf_cls* h, const float* xyz, size_t n, size_t stride, bool idx, bool ground_only = false) {
    if (n > h->c.cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(h->device));
    repack_xyz(xyz, n, stride, h->host);
    const int ni = (int)n;
    if (n) PF_HIP_TRY(hipMemcpyAsync(h->c.pts, h->host.data(), sizeof(float4) * n, hipMemcpyHostToDevice, h->stream));
    PF_HIP_TRY(hipMemcpyAsync(h->d_n, &ni, sizeof(int), hipMemcpyHostToDevice, h->stream));
    cls_enqueue(h->c, h->c.pts, h->d_n, nullptr, nullptr, idx, h->stream, ground_only);
    PF_HIP_TRY(hipGetLastError());
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    return PF_OK;
}
}  // namespace

extern "C" {

void pf_cls_default_params(pf_cls_params* p) {
    if (!p) return;
    p->ground_filter = 1;              // pfilter_kitti.launch:10
    p->gf_min_grid_pts = 8;            // include/preProcess.hpp:575
    p->gf_grid_res = 3.0f;             // :605
    p->gf_max_height_diff = 0.3f;      // :604
    p->gf_neighbor_height_diff = 1.5f; // :603
    p->gf_max_ground_height = 5.0f;    // :601
    p->gf_min_ground_height = -5.0f;   // :602
    p->radius = 1.0f;                  // :703
    p->k = 25;                         // :705
    p->k_min = 8;                      // :706
    p->edge_thre = 0.65f;              // :708
    p->planar_thre = 0.65f;            // :709
    p->linear_vsin_high = 0.94f;       // :710
    p->linear_vsin_low = 0.17f;        // :711
    p->planar_vsin_low = 0.34f;        // :713
    p->beam_h_max = FLT_MAX;           // :714
    p->beam_h_min = 0.5f;              // :715
}

int pf_cls_create(const pf_cls_params* p, int device, size_t max_points, pf_cls** out) {
    if (!out || !cls_params_ok(p) || max_points == 0 || max_points > (size_t)INT_MAX / 2) return PF_EINVAL;
    *out = nullptr;
    int ndev = 0;
    PF_HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(device));
    pf_cls* h = new pf_cls();
    h->device = device;
    h->c.prm = *p;
    int rc = PF_OK;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) rc = PF_EHIP;
    if (rc == PF_OK) rc = cls_alloc(h->c, max_points);
    if (rc == PF_OK && hipMalloc(&h->d_n, sizeof(int)) != hipSuccess) rc = PF_ENOMEM;
    if (rc != PF_OK) {
        pf_cls_destroy(h);
        return rc;
    }
    *out = h;
    return PF_OK;
}

int pf_cls_destroy(pf_cls* h) {
    if (!h) return PF_EINVAL;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    cls_free(h->c);
    (void)hipFree(h->d_n);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return PF_OK;
}

int pf_cls_extract(pf_cls* h, const float* xyz, size_t n, size_t stride_bytes, int32_t* beam, size_t* nb,
                   int32_t* pillar, size_t* np, int32_t* facade, size_t* nf, int32_t* ground, size_t* ng,
                   size_t cap) {
    if (!h || (!xyz && n) || stride_bytes < 12) return PF_EINVAL;
    int rc = cls_run(h, xyz, n, stride_bytes, true);
    if (rc) return rc;
    int cnt[CC_COUNT];
    PF_HIP_TRY(hipMemcpy(cnt, h->c.cnt, sizeof(cnt), hipMemcpyDeviceToHost));
    if (cnt[CC_ERR]) return PF_ECAPACITY;                    // ground grid above kGsMaxCells
    int gerr = 0;
    PF_HIP_TRY(hipMemcpy(&gerr, h->c.grid.err, sizeof(int), hipMemcpyDeviceToHost));
    if (gerr) {
        (void)hipMemset(h->c.grid.err, 0, sizeof(int));
        return PF_ECAPACITY;
    }
    const size_t n0 = (size_t)cnt[CC_CLS], n1 = (size_t)cnt[CC_CLS + 1], n2 = (size_t)cnt[CC_CLS + 2];
    const size_t ngr = (size_t)cnt[CC_NG], nu = (size_t)cnt[CC_NU];
    if (nb) *nb = n0;
    if (np) *np = n1;
    if (nf) *nf = n2;
    if (ng) *ng = ngr;
    if ((beam && n0 > cap) || (pillar && n1 > cap) || (facade && n2 > cap) || (ground && ngr > cap))
        return PF_ECAPACITY;
    if (beam && n0) PF_HIP_TRY(hipMemcpy(beam, h->c.idx_out, sizeof(int) * n0, hipMemcpyDeviceToHost));
    if (pillar && n1) PF_HIP_TRY(hipMemcpy(pillar, h->c.idx_out + n0, sizeof(int) * n1, hipMemcpyDeviceToHost));
    if (facade && n2) PF_HIP_TRY(hipMemcpy(facade, h->c.idx_out + n0 + n1, sizeof(int) * n2, hipMemcpyDeviceToHost));
    if (ground && ngr) PF_HIP_TRY(hipMemcpy(ground, h->c.vals + cnt[CC_NUG], sizeof(int) * ngr, hipMemcpyDeviceToHost));
    (void)nu;
    return PF_OK;
}

int pf_cls_ground_seg(pf_cls* h, const float* xyz, size_t n, size_t stride_bytes, int32_t* ground, size_t* ng,
                      int32_t* unground, size_t* nu, size_t cap) {
    if (!h || (!xyz && n) || stride_bytes < 12) return PF_EINVAL;
    const int gf = h->c.prm.ground_filter;
    h->c.prm.ground_filter = 1;
    int rc = cls_run(h, xyz, n, stride_bytes, false, true);
    h->c.prm.ground_filter = gf;
    if (rc) return rc;
    int cnt[CC_COUNT];
    PF_HIP_TRY(hipMemcpy(cnt, h->c.cnt, sizeof(cnt), hipMemcpyDeviceToHost));
    if (cnt[CC_ERR]) return PF_ECAPACITY;
    const size_t ngr = (size_t)cnt[CC_NG], nun = (size_t)cnt[CC_NU];
    if (ng) *ng = ngr;
    if (nu) *nu = nun;
    if ((ground && ngr > cap) || (unground && nun > cap)) return PF_ECAPACITY;
    if (unground && nun) PF_HIP_TRY(hipMemcpy(unground, h->c.vals, sizeof(int) * nun, hipMemcpyDeviceToHost));
    if (ground && ngr) PF_HIP_TRY(hipMemcpy(ground, h->c.vals + nun, sizeof(int) * ngr, hipMemcpyDeviceToHost));
    return PF_OK;
}

int pf_cls_set_dcvc(pf_cls* h, const pf_dcvc_params* p) {
    if (!h) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->device));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    return cls_set_dcvc(h->c, p);
}

int pf_cls_normals(pf_cls* h, float* normal4, size_t n) {
    if (!h || (!normal4 && n)) return PF_EINVAL;
    int cnt[CC_COUNT];
    PF_HIP_TRY(hipSetDevice(h->device));
    PF_HIP_TRY(hipMemcpy(cnt, h->c.cnt, sizeof(cnt), hipMemcpyDeviceToHost));
    if (n > (size_t)cnt[CC_NU]) return PF_ECAPACITY;
    if (n) PF_HIP_TRY(hipMemcpy(normal4, h->c.nrm, sizeof(float4) * n, hipMemcpyDeviceToHost));
    return PF_OK;
}

int pf_cls_classify(pf_cls* h, const float* xyz, size_t n, size_t stride_bytes, uint8_t* cls, int32_t* pt_num) {
    if (!h || (!xyz && n) || stride_bytes < 12) return PF_EINVAL;
    const int gf = h->c.prm.ground_filter;
    DcvcGPU* dc = h->c.dcvc;                          // featureExtract alone: no ground_seg, no DCVC
    h->c.prm.ground_filter = 0;
    h->c.dcvc = nullptr;
    int rc = cls_run(h, xyz, n, stride_bytes, false);
    h->c.prm.ground_filter = gf;
    h->c.dcvc = dc;
    if (rc) return rc;
    int gerr = 0;
    PF_HIP_TRY(hipMemcpy(&gerr, h->c.grid.err, sizeof(int), hipMemcpyDeviceToHost));
    if (gerr) {
        (void)hipMemset(h->c.grid.err, 0, sizeof(int));
        return PF_ECAPACITY;
    }
    if (cls && n) PF_HIP_TRY(hipMemcpy(cls, h->c.code, n, hipMemcpyDeviceToHost));
    if (pt_num && n) PF_HIP_TRY(hipMemcpy(pt_num, h->c.ptnum, sizeof(int) * n, hipMemcpyDeviceToHost));
    return PF_OK;
}

}  // extern "C"
