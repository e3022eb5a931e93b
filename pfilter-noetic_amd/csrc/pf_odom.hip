// Device-resident odometry: Odom_ES_EstimationClass::updatePointsToMap / initMapWithPoints
// (src/odomEstimationClass.cpp:217-282) as a fixed sequence of launches with every count kept on
// the device, so a frame is enqueued without any host round trip (and can be replayed as a graph).
//
//   PredictTail      constant-velocity prediction, optimization_count schedule, map-size gate (:232-247),
//                    as the tail of the grid-bounds kernel
//   VoxelGrid        k_vg_minmax / k_vg_keys / radix sort / segments / k_vg_reduce: PCL 1.10 VoxelGrid
//                    (edge leaf 0.4, surf 0.8, :242-245) for both clouds in one batched pass
//   grid_build       1 m cell grids of the edge and surf maps (the kd-trees of :249-250)
//   per outer iteration (:252-272)
//     k_assoc        pointAssociateToMap + exact 5-NN + line fit (eigen, :299-331) / plane fit (QR,
//                    :447-476) + round / sparsity
//     p-index        (neighbour, query) pairs radix-sorted by neighbour: c_i(n) = earlier valid queries
//                    sharing neighbour n reproduces the in-order increments of :345-346 / :493-496
//     k_observe      observe/round skip test (:348-356, :497-505), kept flags, weight statistics
//     k_lm_solve     one workgroup runs Ceres 1.14 LM (Huber 0.1, Jacobi scaling, radius 1e4,
//                    <= 4 iterations) on the 6x6 normal equations, all iterations in one launch
//   k_finalize       odom from the solved pose (:278-280), pose output (node: copy.cpp:105-107)
//   addPointsToMap   transform/append, CropBox +-100 m, rgbds (centroid + max r/g), extractstablepoint,
//                    ageing (:589-647): batched keys / radix sort / segments / reduce / compaction
#include "pf_odom.h"
#include "pf_geom.h"

#include <climits>
#include <cmath>
#include <cstdlib>
#include <vector>
#include <cstring>

#ifndef PF_TIE_LEVELS_A
#define PF_TIE_LEVELS_A 0   // big levels of the tie-order VoxelGrid sort (0: classes straight to k_tie_medium)
#endif
#ifndef PF_TIE_LEVELS_B
#define PF_TIE_LEVELS_B 0   // least big levels of the tie-order rgbds sort
#endif

namespace pf {
namespace {

constexpr u32 kSentinel = 0xFFFFFFFFu;
struct VgLeaf {                        // per-class leaf sizes
    float v[kMaxC];
    __device__ __forceinline__ float at(int c) const { return c == 0 ? v[0] : (c == 1 ? v[1] : v[2]); }
};
#ifndef PF_GRID
#define PF_GRID 512
#endif
constexpr int kGrid = PF_GRID;   // grid-stride workgroups for per-point kernels

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
__device__ __forceinline__ u32 w_r(const float4& p) { return __float_as_uint(p.w) & 255u; }
__device__ __forceinline__ u32 w_g(const float4& p) { return (__float_as_uint(p.w) >> 8) & 255u; }

__device__ __forceinline__ iso load_iso(const double* R, const double* t) {
    iso a;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) a.R.m[i][j] = R[3 * i + j];
    a.t = d3{t[0], t[1], t[2]};
    return a;
}
__device__ __forceinline__ void store_iso(const iso& a, double* R, double* t) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = a.R.m[i][j];
    t[0] = a.t.x; t[1] = a.t.y; t[2] = a.t.z;
}

// pointAssociateToMap (:162-174): double transform, float result
__device__ __forceinline__ float4 associate(const double* prm, float4 p) {
    const qd q{prm[0], prm[1], prm[2], prm[3]};
    const d3 w = add3(qrot(q, d3{(double)p.x, (double)p.y, (double)p.z}), d3{prm[4], prm[5], prm[6]});
    return make_float4((float)w.x, (float)w.y, (float)w.z, p.w);
}

// per-class values picked with selects: a per-lane class index into an array would put the array
// in scratch memory
template <class T>
__device__ __forceinline__ T sel3(int c, T a, T b, T d) { return c == 0 ? a : (c == 1 ? b : d); }

// per-class pointer sets passed by value (kernel arguments)
struct Clouds {
    const float4* p[kMaxC];
    __device__ __forceinline__ const float4* at(int c) const { return sel3(c, p[0], p[1], p[2]); }
};
struct CloudsW {
    float4* p[kMaxC];
    __device__ __forceinline__ float4* at(int c) const { return sel3(c, p[0], p[1], p[2]); }
};

// a concatenation of per-class ranges: element i belongs to class cls(i) at local index i - start(c)
template <int NC>
struct CatIdx {
    int end[kMaxC];
    __device__ __forceinline__ int total() const { return end[NC - 1]; }
    __device__ __forceinline__ int cls(int i) const {
        return NC == 2 ? (i < end[0] ? 0 : 1) : (i < end[0] ? 0 : (i < end[1] ? 1 : 2));
    }
    __device__ __forceinline__ int start(int c) const { return c == 0 ? 0 : (c == 1 ? end[0] : end[1]); }
};
template <int NC>
__device__ __forceinline__ CatIdx<NC> cat_idx(const int* counts) {
    CatIdx<NC> x;
    int acc = 0;
#pragma unroll
    for (int k = 0; k < kMaxC; ++k) {
        acc += k < NC ? counts[k] : 0;
        x.end[k] = acc;
    }
    return x;
}

// per-class float min/max of xyz reduced over the workgroup, one atomic per value and workgroup;
// v[6 c + k]: min (k < 3) / max (k >= 3) of class c
__device__ __forceinline__ void minmax_commit(float (&v)[6 * kMaxC], u32* acc, int nc) {
    __shared__ float red[4][6 * kMaxC];
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 6 * kMaxC; ++k) {
        if (k >= 6 * nc) break;                    // uniform: classes the handle does not have
        const float r = ((k % 6) < 3) ? wave_minf(v[k]) : wave_maxf(v[k]);
        if (lane_id() == 0) red[w][k] = r;
    }
    __syncthreads();
    if (threadIdx.x < 6 * nc) {
        const int k = threadIdx.x;
        float r = red[0][k];
        for (int ww = 1; ww < 4; ++ww) r = ((k % 6) < 3) ? fminf(r, red[ww][k]) : fmaxf(r, red[ww][k]);
        const bool any = ((k % 6) < 3) ? (r != FLT_MAX) : (r != -FLT_MAX);
        if (any) {
            if ((k % 6) < 3) atomicMin(&acc[k], f2ord(r));
            else atomicMax(&acc[k], f2ord(r));
        }
    }
}
// branch-free per class (a branch per class lets the compiler turn v[] into a scratch array indexed
// by the class)
__device__ __forceinline__ void minmax_add(float (&v)[6 * kMaxC], int c, float4 p) {
    const float xyz[3] = {p.x, p.y, p.z};
#pragma unroll
    for (int cc = 0; cc < kMaxC; ++cc) {
        const bool mine = cc == c;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            v[6 * cc + k] = mine ? fminf(v[6 * cc + k], xyz[k]) : v[6 * cc + k];
            v[6 * cc + 3 + k] = mine ? fmaxf(v[6 * cc + 3 + k], xyz[k]) : v[6 * cc + 3 + k];
        }
    }
}
__device__ __forceinline__ void minmax_init(float (&v)[6 * kMaxC]) {
#pragma unroll
    for (int k = 0; k < 6 * kMaxC; ++k) v[k] = ((k % 6) < 3) ? FLT_MAX : -FLT_MAX;
}

// ---------------------------------------------------------------------------------------------
// copies the stage slots a frame's odometry reads from its pipeline slot's counters
__device__ __forceinline__ void pull_stage_counts(int* cnt, const int* scnt) {
    cnt[C_NIN] = scnt[C_NIN];
    cnt[C_VGN] = scnt[C_VGN];
    cnt[C_NQ] = scnt[C_NQ];
    for (int c = 0; c < kMaxC; ++c) {
        cnt[C_IN + c] = scnt[C_IN + c];
        cnt[C_DS + c] = scnt[C_DS + c];
    }
}

__global__ void k_pull_counts(int* __restrict__ cnt, const int* __restrict__ scnt) {
    if (threadIdx.x == 0) pull_stage_counts(cnt, scnt);
}

// constant-velocity prediction, optimization_count schedule, map-size gate (:232-247); thread 0's
// chain, thread < 18 reset the map-update bounds. Runs on an extra workgroup of the grid-bounds kernel.
struct PredictTail {
    static constexpr bool kActive = true;
    DevState* st;
    int* cnt;
    const int* scnt;
    u32* acc;
    ClassCfg cls;
    __device__ void operator()(int t) const {
        if (t < 6 * kMaxC) acc[A_RG + t] = ((t % 6) < 3) ? 0xFFFFFFFFu : 0u;   // map-update bounds
        if (t != 0) return;
        pull_stage_counts(cnt, scnt);
        if (st->optimization_count > 2) st->optimization_count--;                 // :232-233
        const iso odom = load_iso(st->odomR, st->odomt);
        const iso last = load_iso(st->lastR, st->lastt);
        const iso pred = iso_mul(odom, iso_mul(iso_inv(last), odom));             // :235
        store_iso(odom, st->lastR, st->lastt);
        store_iso(pred, st->odomR, st->odomt);
        const qd q = m2q(polar_rotation(pred.R));                                  // :239 (Eigen 3.3 rotation())
        st->params[0] = q.x; st->params[1] = q.y; st->params[2] = q.z; st->params[3] = q.w;
        st->params[4] = pred.t.x; st->params[5] = pred.t.y; st->params[6] = pred.t.z;
        int gate = 1;                              // :247 / BPF :721: line maps > 10, plane maps > 50
        for (int c = 0; c < cls.nc; ++c) gate &= cnt[C_M + c] > (cls.is_plane(c) ? 50 : 10) ? 1 : 0;
        st->gate = gate;
        cnt[C_GATE] = gate;
        cnt[C_OUTER] = gate ? st->optimization_count : 0;
        cnt[C_LM_ITERS] = 0;
        for (int c = 0; c < kMaxC; ++c) cnt[C_KEPT + c] = cnt[C_VALID + c] = 0;
    }
};

// the first kernel of an update whose grid dims k_rgm_finish computed (OdomGPU::dims_fresh): the
// count reads dims_next; its tail workgroup copies them into the grid (read by the scan, the placement
// and the kNN, all later kernels) and runs the pose prediction
struct FreshTail {
    static constexpr bool kActive = true;
    PredictTail pred;
    const int* dims_next;
    int* dims;
    int* d_ncells;
    __device__ void operator()(int t) const {
        if (t < 8 * kGridMaps) dims[t] = dims_next[t];
        if (t == 8 * kGridMaps) *d_ncells = dims_next[t];
        pred(t);
    }
};

// voxel-grid stage set-up (stream A): reset the min/max accumulators, batch size
__global__ void k_vg_begin(int* __restrict__ scnt, u32* __restrict__ acc, int nc) {
    const int t = threadIdx.x;
    if (t < 6 * kMaxC) acc[A_VG + t] = ((t % 6) < 3) ? 0xFFFFFFFFu : 0u;
    if (t == 0) {
        int n = 0;
        for (int c = 0; c < nc; ++c) n += scnt[C_IN + c];
        scnt[C_VGN] = n;
    }
}

// ----------------------------------- VoxelGrid (B.1) ------------------------------------------
template <int NC>
__global__ void __launch_bounds__(256) k_vg_minmax(Clouds in, const int* __restrict__ cnt, u32* __restrict__ acc) {
    constexpr int nc = NC;
    const CatIdx<NC> ci = cat_idx<NC>(cnt + C_IN);
    float v[6 * kMaxC];
    minmax_init(v);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ci.total(); i += gridDim.x * blockDim.x) {
        const int c = ci.cls(i);
        minmax_add(v, c, in.at(c)[i - ci.start(c)]);
    }
    minmax_commit(v, acc + A_VG, nc);
}

// keys: class in bits 30-31, the voxel index below (sorted by class, then voxel)
template <int NC>
__global__ void __launch_bounds__(256) k_vg_keys(Clouds in, const int* __restrict__ cnt, const u32* __restrict__ acc,
                                                  VgLeaf leaf, u32* __restrict__ keys, u32* __restrict__ vals,
                                                  SortHist sh) {
    __shared__ u32 lh[4][256];
    sort_hist_begin(lh);
    const CatIdx<NC> ci = cat_idx<NC>(cnt + C_IN);
    const int n = ci.total();
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int c = ci.cls(i);
        const float4 p = in.at(c)[i - ci.start(c)];
        const float inv = 1.0f / leaf.at(c);                      // inverse_leaf_size_
        const u32* a = acc + A_VG + 6 * c;
        const float mn[3] = {ord2f(a[0]), ord2f(a[1]), ord2f(a[2])};
        const float mx[3] = {ord2f(a[3]), ord2f(a[4]), ord2f(a[5])};
        const long long dx = (long long)((mx[0] - mn[0]) * inv) + 1;
        const long long dy = (long long)((mx[1] - mn[1]) * inv) + 1;
        const long long dz = (long long)((mx[2] - mn[2]) * inv) + 1;
        u32 key;
        if (dx * dy * dz > (long long)INT_MAX) {
            key = (u32)(i - ci.start(c));        // "leaf too small": output = input, order kept
        } else {
            int minb[3], div[3];
            for (int k = 0; k < 3; ++k) {
                minb[k] = (int)floorf(mn[k] * inv);
                div[k] = (int)floorf(mx[k] * inv) - minb[k] + 1;
            }
            const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
            const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
            const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
            key = (u32)(i0 + i1 * div[0] + i2 * (div[0] * div[1]));
        }
        key = (key & 0x3fffffffu) | ((u32)c << 30);
        keys[i] = key;
        vals[i] = (u32)i;
        sort_hist_add(lh, key, sh.passes);
    }
    sort_hist_end(lh, sh, n, n);
}

// One wave per voxel: the lanes gather up to 512 members at a time into the wave's LDS buffer, then
// lanes 0, 1, 2 run the x, y, z sums over them in sorted (stable) order, one LDS read and one f32
// add per member, so the order of additions is PCL's sequential one (the chain of the largest voxel
// is the kernel's critical path: a few hundred ground points under the sensor at the surf leaf)
__device__ __forceinline__ float lane_f(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}
template <int NC>
__global__ void __launch_bounds__(256) k_vg_reduce(Clouds in, const u32* __restrict__ keys, const u32* __restrict__ vals,
                                                    const u32* __restrict__ segstart, int* __restrict__ cnt,
                                                    CloudsW ds) {
    __shared__ float mem[4][8 * 64 * 4];                 // per wave: 512 members, x y z w
    constexpr int nc = NC;
    const CatIdx<NC> ci = cat_idx<NC>(cnt + C_IN);
    const int n = cnt[C_VGN];
    const int nseg = cnt[C_NSEG];
    const int nlt0 = cnt[C_NLT], nlt1 = cnt[C_NLT + 1];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        cnt[C_DS] = nlt0;
        cnt[C_DS + 1] = nc > 1 ? nlt1 - nlt0 : 0;
        cnt[C_DS + 2] = nc > 2 ? nseg - nlt1 : 0;
        cnt[C_NQ] = nseg;
    }
    const int l = lane_id();
    float* wm = mem[threadIdx.x >> 6];
    const int waves = gridDim.x * (blockDim.x >> 6);
    for (int sg = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; sg < nseg; sg += waves) {
        const u32 b0 = segstart[sg], b1 = (sg + 1 < nseg) ? segstart[sg + 1] : (u32)n;
        const int c = (int)(keys[b0] >> 30);
        const float4* src = in.at(c);
        const int s0 = ci.start(c);
        float acc = 0.f;                                    // lane k < 3: the sum of component k
        for (u32 base = b0; base < b1; base += 8 * 64) {   // AccumulatorXYZ, sorted (stable) order
            u32 idx[8];                                     // up to 512 members in flight at once
            float4 p[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) idx[u] = base + u * 64 + l < b1 ? vals[base + u * 64 + l] : 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                p[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (idx[u] != 0xFFFFFFFFu) p[u] = src[(int)idx[u] - s0];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) reinterpret_cast<float4*>(wm)[u * 64 + l] = p[u];
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const int m = (int)min(512u, b1 - base);
            if (l < 3) {
                int j = 0;
                for (; j + 4 <= m; j += 4) {               // reads run ahead of the dependent adds
                    const float a0 = wm[4 * j + l], a1 = wm[4 * (j + 1) + l];
                    const float a2 = wm[4 * (j + 2) + l], a3 = wm[4 * (j + 3) + l];
                    acc += a0;
                    acc += a1;
                    acc += a2;
                    acc += a3;
                }
                for (; j < m; ++j) acc += wm[4 * j + l];
            }
            __builtin_amdgcn_wave_barrier();               // the buffer is refilled by the next round
        }
        const float sx = lane_f(acc, 0), sy = lane_f(acc, 1), sz = lane_f(acc, 2);
        if (l == 0) {
            const float nn = (float)(b1 - b0);
            // rgb of inputs is 0 (copyPointCloud XYZI -> XYZRGB): averages stay 0
            const float4 o = make_float4(sx / nn, sy / nn, sz / nn, __uint_as_float(0u));
            ds.at(c)[sg - (c == 0 ? 0 : (c == 1 ? nlt0 : nlt1))] = o;
        }
    }
}

// ---------------------------------- association ---------------------------------------------
struct AssocArgs {
    const DevState* st;
    int* cnt;
    u32* acc;
    GridView gv;
    ClassCfg cls;
    Clouds ds;
    Clouds map;
    int* nbr;
    int* qflag;
    double* geo;
    float* spars;
    float* roundv;
    int4* pbkt;            // p-index buckets (one per map point, class c's at c * map_cap)
    int* pnext;
    u32 map_cap;
    u32* lm_arrive;
    double* lm_part;       // [kLmEvals][kLmBlocks][32] LM partials, reset to kPartSentinel here
};

// line fit (:302-331) / plane fit (:449-476), round and sparsity, p-index pair keys of query q
__device__ __forceinline__ void assoc_fit(const AssocArgs& a, int q, int c, const int* id, int found) {
    bool valid = false;
    const float4* mp = a.map.at(c);
    if (found == 5) {
        double px[5], py[5], pz[5];
        u32 rsum = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const float4 m = mp[id[j]];
            px[j] = m.x; py[j] = m.y; pz[j] = m.z;
            rsum += w_r(m);
        }
        double* G = a.geo + 8 * (size_t)q;
        if (!a.cls.is_plane(c)) {                                // :302-331 (BPF beam / pillar :775-804)
            d3 center{0, 0, 0};
            for (int j = 0; j < 5; ++j) center = add3(center, d3{px[j], py[j], pz[j]});
            center = d3{center.x / 5.0, center.y / 5.0, center.z / 5.0};
            double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
            for (int j = 0; j < 5; ++j) {
                const double tv[3] = {px[j] - center.x, py[j] - center.y, pz[j] - center.z};
                for (int r = 0; r < 3; ++r)
                    for (int cc = 0; cc < 3; ++cc) cov[r][cc] = cov[r][cc] + tv[r] * tv[cc];
            }
            double ev[3], V[3][3];
#ifndef PF_DEV_NOEIG
            eig3(cov, ev, V);
#else
            for (int i = 0; i < 3; ++i) { ev[i] = cov[i][i] * (i + 1); for (int j = 0; j < 3; ++j) V[i][j] = cov[i][j]; }
#endif
            if (ev[2] > 3 * ev[1]) {
                valid = true;
                const d3 dir{V[0][2], V[1][2], V[2][2]};
                G[0] = 0.1 * dir.x + center.x; G[1] = 0.1 * dir.y + center.y; G[2] = 0.1 * dir.z + center.z;
                G[3] = -0.1 * dir.x + center.x; G[4] = -0.1 * dir.y + center.y; G[5] = -0.1 * dir.z + center.z;
            }
        } else {                                                 // :449-476 (BPF facade :1070-1104)
            double A[5][3];
            for (int j = 0; j < 5; ++j) { A[j][0] = px[j]; A[j][1] = py[j]; A[j][2] = pz[j]; }
#ifndef PF_DEV_NOQR
            d3 n = plane5(A);
#else
            d3 n{A[0][0] * 0.01, A[1][1] * 0.01, 1.0 + A[2][2] * 1e-9};
#endif
            const double nd = 1 / nrm3(n);
            const double z = n.x * n.x + n.y * n.y + n.z * n.z;
            if (z > 0.0) {
                const double sq = sqrt(z);
                n = d3{n.x / sq, n.y / sq, n.z / sq};
            }
            valid = true;
            for (int j = 0; j < 5; ++j)
                if (fabs(n.x * px[j] + n.y * py[j] + n.z * pz[j] + nd) > 0.2) { valid = false; break; }
            if (valid) {
                G[0] = n.x; G[1] = n.y; G[2] = n.z;
                G[3] = (double)(float)nd;                        // surfInfo::negative_OA_dot_norm is float (A.7)
            }
        }
        if (valid) {
            a.roundv[q] = (float)(rsum / 5.0);                   // :339-344 (r constant within a frame)
            d3 cn{0, 0, 0};                                      // sparsity, :367-385
            for (int j = 0; j < 5; ++j) cn = add3(cn, d3{px[j], py[j], pz[j]});
            cn = d3{cn.x / 5, cn.y / 5, cn.z / 5};
            float sum = 0;
            for (int j = 0; j < 5; ++j) sum += nrm3(sub3(cn, d3{px[j], py[j], pz[j]}));
            sum /= 5.0;
            a.spars[q] = sum;
        }
    }
    a.qflag[q] = valid ? 1 : 0;
#ifdef PF_DEV_NOPUSH
    if (false) {
#else
    if (valid) {               // p-index: push the 5 pairs onto their map points' lists (:345-346, :493-496)
#endif
        const u32 off = (u32)c * a.map_cap;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            int* b = reinterpret_cast<int*>(a.pbkt + (size_t)kBktQuads * (off + (u32)id[j]));
            const int p = 5 * q + j;
            const int slot = atomicAdd(&b[0], 1);                  // {count, kBktInline pairs, overflow head}
            if (slot < kBktInline) b[1 + slot] = p;
            else a.pnext[p] = atomicExch(&b[kBktHead], p);
        }
    }
}

// pointAssociateToMap + exact 5-NN (a team of T lanes per query, :297-300, :445-448), then the fit on
// the team's first lane, which pushes the query's pairs into the p-index buckets. The team size
// follows the frame's query count (uniform over the grid, so every wave takes the same branch): 16
// lanes up to kAssocWideMax queries, 8 above. End of round 2, frames/s with teams of 8 / 16 / 32: S64
// (~6k queries) 3781 / 3843 / 3563; the dense S64V scene (~10k) 3726 / 3645 with 8 / 16.
#ifndef PF_ASSOC_WIDE_MAX
#define PF_ASSOC_WIDE_MAX 8192
#endif
constexpr int kAssocWideMax = PF_ASSOC_WIDE_MAX;
template <int NC, int T>
__device__ __forceinline__ void assoc_queries(const AssocArgs& a, const CatIdx<NC>& qi, int nq, const double* prm) {
    static_assert(T >= 5, "k_assoc writes the 5 neighbours from 5 lanes of the team");
    const int tl = lane_id() & (T - 1);
    const int teams = gridDim.x * (blockDim.x / T);
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int team = gt / T, wave_team0 = (gt & ~63) / T;
    for (int off = 0; wave_team0 + off < nq; off += teams) {     // trip count uniform per wave
        const int q0 = team + off;
        const bool active = q0 < nq;
        const int c = active ? qi.cls(q0) : 0;
        float4 pw = make_float4(0.f, 0.f, 0.f, 0.f);
        if (active) pw = associate(prm, a.ds.at(c)[q0 - qi.start(c)]);
        float d[5];
        int id[5];
        const int found = knn5_team<T>(a.gv, c, pw.x, pw.y, pw.z, active, d, id);
        if (active && tl < 5) {                                  // neighbours, read again by k_observe
            int iv = id[0];
#pragma unroll
            for (int k = 1; k < 5; ++k)
                if (tl == k) iv = id[k];
            a.nbr[5 * q0 + tl] = found == 5 ? iv : -1;
        }
#ifndef PF_DEV_NOFIT
        if (active && tl == 0) assoc_fit(a, q0, c, id, found);
#else
        if (active && tl == 0) a.qflag[q0] = 0;                  // development: time the kNN alone
#endif
    }
}
template <int NC>
__global__ void __launch_bounds__(256) k_assoc(AssocArgs a) {
    const CatIdx<NC> qi = cat_idx<NC>(a.cnt + C_DS);
    const int nq = a.cnt[C_NQ];
    const int gate = a.st->gate;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int k = 0; k < kLmEvalSlots; ++k) a.lm_arrive[k] = 0u;       // LM claim masks
        a.cnt[C_NPAIR] = gate ? 5 * nq : 0;
        for (int c = 0; c < kMaxC; ++c) a.cnt[C_KEPT + c] = a.cnt[C_VALID + c] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x < 4 * kMaxC) a.acc[A_W + threadIdx.x] = (threadIdx.x & 1) ? 0u : 0xFFFFFFFFu;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kLmEvals * kLmBlocks * 32; i += gridDim.x * blockDim.x)
        reinterpret_cast<unsigned long long*>(a.lm_part)[i] = kPartSentinel;   // LM partials: none published
    if (!gate) {                                   // solve skipped: no association is valid
        for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) a.qflag[q] = 0;
        return;                                    // (no pairs: every block leaves before the prologue)
    }
    double prm[7];
    for (int k = 0; k < 7; ++k) prm[k] = a.st->params[k];
    if (nq <= kAssocWideMax) assoc_queries<NC, 16>(a, qi, nq, prm);
    else assoc_queries<NC, 8>(a, qi, nq, prm);
}

// ---- association kNN probe (pf_odom_probe_assoc): k_assoc's kNN alone on the last frame ---------
// The queries of the last frame (its down-sampled points through the solved pose), the same grid and
// the same team search as k_assoc, neighbours into scratch: nothing of the estimator's state changes.
template <int NC, int T>
__device__ __forceinline__ void assoc_probe(const DevState* __restrict__ st, const int* __restrict__ cnt, GridView gv,
                                            Clouds ds, int* __restrict__ nbr, float4* __restrict__ qout) {
    const CatIdx<NC> qi = cat_idx<NC>(cnt + C_DS);
    const int nq = cnt[C_NQ];
    double prm[7];
    for (int k = 0; k < 7; ++k) prm[k] = st->params[k];
    const int tl = lane_id() & (T - 1);
    const int teams = gridDim.x * (blockDim.x / T);
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int team = gt / T, wave_team0 = (gt & ~63) / T;
    for (int off = 0; wave_team0 + off < nq; off += teams) {
        const int q0 = team + off;
        const bool active = q0 < nq;
        const int c = active ? qi.cls(q0) : 0;
        float4 pw = make_float4(0.f, 0.f, 0.f, 0.f);
        if (active) pw = associate(prm, ds.at(c)[q0 - qi.start(c)]);
        float d[5];
        int id[5];
        const int found = knn5_team<T>(gv, c, pw.x, pw.y, pw.z, active, d, id);
        if (active && tl == 0) {
            nbr[q0] = found == 5 ? id[4] : -1;
            if (qout) qout[q0] = make_float4(pw.x, pw.y, pw.z, __int_as_float(c));
        }
    }
}

template <int NC>
__global__ void __launch_bounds__(256) k_assoc_probe_t16(const DevState* st, const int* cnt, GridView gv, Clouds ds,
                                                          int* nbr, float4* qout) {
    assoc_probe<NC, 16>(st, cnt, gv, ds, nbr, qout);
}
template <int NC>
__global__ void __launch_bounds__(256) k_assoc_probe_t8(const DevState* st, const int* cnt, GridView gv, Clouds ds,
                                                         int* nbr, float4* qout) {
    assoc_probe<NC, 8>(st, cnt, gv, ds, nbr, qout);
}

// SURVEY 8(d)'s algorithmic bytes of those queries: 16 + 40 + 27 x 8 + 16 |C(q)| each, |C(q)| = the
// map points in the 27 cells of the query's class grid around its cell
template <int NC>
__global__ void __launch_bounds__(256) k_assoc_cellpop(const DevState* __restrict__ st, const int* __restrict__ cnt,
                                                        GridView gv, Clouds ds, unsigned long long* __restrict__ out) {
    const CatIdx<NC> qi = cat_idx<NC>(cnt + C_DS);
    const int nq = cnt[C_NQ];
    double prm[7];
    for (int k = 0; k < 7; ++k) prm[k] = st->params[k];
    unsigned long long acc = 0;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
        const int c = qi.cls(q);
        const float4 pw = associate(prm, ds.at(c)[q - qi.start(c)]);
        const int* dm = gv.dims + 8 * c;
        unsigned long long pop = 0;
        if (dm[7]) {
            const int cx = (int)floorf(pw.x), cy = (int)floorf(pw.y), cz = (int)floorf(pw.z);
            for (int oz = -1; oz <= 1; ++oz)
                for (int oy = -1; oy <= 1; ++oy) {
                    const int y = cy + oy - dm[1], z = cz + oz - dm[2];
                    if (y < 0 || y >= dm[4] || z < 0 || z >= dm[5]) continue;
                    const int x0 = max(cx - 1 - dm[0], 0), x1 = min(cx + 1 - dm[0], dm[3] - 1);
                    if (x0 > x1) continue;
                    const int row = dm[6] + (z * dm[4] + y) * dm[3];
                    pop += gv.cell_start[row + x1 + 1] - gv.cell_start[row + x0];
                }
        }
        acc += 16ull + 40ull + 27ull * 8ull + 16ull * pop;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane_id() == 0 && acc) atomicAdd(out, acc);
}

struct ObsArgs {
    int* cnt;
    u32* acc;
    ClassCfg cls;
    Clouds map;
    CloudsW ds;
    const int* nbr;
    int* qflag;
    const int4* pbkt;
    const int* pnext;
    u32* tailinc;
    u32 map_cap;
    const float* roundv;
    const float* spars;
    float* observe;
    int k_new;             // the edge and surf thresholds are equal (init :198-205, BPF :668-674)
    float theta_p;
    int theta_max;
    int* err;              // sticky error word E_LM
};

// observeMean / the skip test of one query (:332-356, :480-505), reads only: its pairs' ranks in their
// map points' p-index buckets, the observe value and the skip decision (applied by observe_commit)
struct ObsRes {
    int f;                 // qflag: bit 0 valid association
    int c;
    bool skip;
    float observe, round;
    u32 tinc[5];           // p-index increments carried by the query's pairs (k_lm_solve applies them)
};
template <int NC>
__device__ __forceinline__ void observe_eval(const ObsArgs& a, const CatIdx<NC>& qi, int nq, int q, ObsRes& r) {
    // the flag and the five neighbours are read together (one memory round trip: the neighbours of an
    // invalid query are in bounds and unused), then the buckets and the neighbours' g bytes together
    r.f = a.qflag[q];
    int nb[5], cur[5], rank[5], len[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) nb[j] = a.nbr[5 * q + j];
    r.c = 0;
    r.skip = true;
    r.observe = r.round = 0.f;
#pragma unroll
    for (int j = 0; j < 5; ++j) r.tinc[j] = 0u;
    if (!(r.f & 1)) return;
    const int c = qi.cls(q);
    r.c = c;
    const float4* mp = a.map.at(c);
    // c_i(n) = valid queries before q sharing neighbour n: count the smaller pair ids in n's bucket
    // (filled in any order by k_assoc: kBktInline pairs inline, the rest on an overflow list); the pair
    // with the largest id carries n's increment
    int4 bk[5][kBktQuads];                               // every bucket read at once
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int k = 0; k < kBktQuads; ++k) bk[j][k] = a.pbkt[(size_t)kBktQuads * ((u32)c * a.map_cap + (u32)nb[j]) + k];
    u32 g0[5];                                           // the g bytes (nothing writes them in this pass)
#pragma unroll
    for (int j = 0; j < 5; ++j) g0[j] = w_g(mp[nb[j]]);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int p = 5 * q + j;
        const int* w = reinterpret_cast<const int*>(bk[j]);
        len[j] = w[0];
        rank[j] = 0;
#pragma unroll
        for (int k = 0; k < kBktInline; ++k) rank[j] += (w[0] > k && w[1 + k] < p) ? 1 : 0;
        cur[j] = w[0] > kBktInline ? w[kBktHead] : -1;
#ifdef PF_DEV_NOCHAIN
        cur[j] = -1;                                     // development: time without the list walks
#endif
    }
    for (int step = 0;; ++step) {
        bool more = false;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            if (cur[j] < 0) continue;
            rank[j] += cur[j] < 5 * q + j ? 1 : 0;
            cur[j] = a.pnext[cur[j]];
            more |= cur[j] >= 0;
        }
        if (!more) break;
        if (step > 5 * nq) { a.cnt[C_ERR] = 1; atomicOr(a.err, 2); break; }   // a list longer than every pair: corrupt
    }
    int gs = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        gs += min(255u, g0[j] + (u32)rank[j]);
        r.tinc[j] = rank[j] == len[j] - 1 ? (u32)len[j] : 0u;
    }
    float observe = gs / 5.0 + 1;                        // :332-338 / :480-486
    const float round = a.roundv[q];
    if (observe / round > 5) observe = 255;              // :348-349
    r.skip = observe < round * a.theta_p && round > a.k_new && observe < a.theta_max;   // :350-353
    r.observe = observe;
    r.round = round;
}
// the query's outputs: pair increments, and for a kept residual the kept bit, observe and the r / g
// bytes of its down-sampled point (:354-355). shared: the kept bit and the r / g word are read by other
// workgroups of the same launch (k_lm_solve with the observe pass fused), so they are written through
// (agent-scope atomic stores)
template <int NC>
__device__ __forceinline__ void observe_commit(const ObsArgs& a, const CatIdx<NC>& qi, int q, const ObsRes& r,
                                               bool shared) {
#pragma unroll
    for (int j = 0; j < 5; ++j) a.tailinc[5 * q + j] = r.tinc[j];
    if (!(r.f & 1) || r.skip) return;
    const u32 rq = (u32)min(255, int(r.round)), gq = (u32)min(255, int(r.observe));
    float* wp = &a.ds.at(r.c)[q - qi.start(r.c)].w;
    a.observe[q] = r.observe;
    if (shared) {
        __hip_atomic_store(&a.qflag[q], r.f | 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(reinterpret_cast<u32*>(wp), pack_rg(rq, gq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        a.qflag[q] = r.f | 2;
        *wp = __uint_as_float(pack_rg(rq, gq));
    }
}

template <int NC>
__global__ void __launch_bounds__(256) k_observe(ObsArgs a) {
    const CatIdx<NC> qi = cat_idx<NC>(a.cnt + C_DS);
    const int nq = a.cnt[C_NQ];
    const int t = threadIdx.x;
    float mn[kMaxC][2], mx[kMaxC][2];
    int nvalid[kMaxC], nkept[kMaxC];
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
        mn[c][0] = mn[c][1] = FLT_MAX;
        mx[c][0] = mx[c][1] = -FLT_MAX;
        nvalid[c] = nkept[c] = 0;
    }
    for (int q = blockIdx.x * blockDim.x + t; q < nq; q += gridDim.x * blockDim.x) {
        ObsRes r;
        observe_eval<NC>(a, qi, nq, q, r);
        observe_commit<NC>(a, qi, q, r, false);
        if (!(r.f & 1)) continue;
        const float sp = a.spars[q];
        const bool skip = r.skip;
        const float observe = r.observe;
        const int c = r.c;
#pragma unroll
        for (int cc = 0; cc < kMaxC; ++cc) {                  // static indices (registers, not scratch)
            if (cc != c) continue;
            ++nvalid[cc];
            if (skip) continue;
            ++nkept[cc];
            mn[cc][0] = fminf(mn[cc][0], observe); mx[cc][0] = fmaxf(mx[cc][0], observe);
            mn[cc][1] = fminf(mn[cc][1], sp); mx[cc][1] = fmaxf(mx[cc][1], sp);
        }
    }
    // workgroup totals, then one atomic per statistic and workgroup (not per wave):
    // v[2 c] valid, v[2 c + 1] kept, v[2 kMaxC + 4 c + 2 ww (+ 1)] min (max) of observe / sparsity
    constexpr int NV = 6 * kMaxC;
    __shared__ u32 wred[4][NV];
    const int w = t >> 6;
    constexpr int nc = NC;
    u32 v[NV];
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
        if (c >= nc) {                             // uniform: classes the handle does not have
            v[2 * c] = v[2 * c + 1] = 0u;
#pragma unroll
            for (int ww = 0; ww < 2; ++ww) {
                v[2 * kMaxC + 4 * c + 2 * ww] = f2ord(FLT_MAX);
                v[2 * kMaxC + 4 * c + 2 * ww + 1] = f2ord(-FLT_MAX);
            }
            continue;
        }
        v[2 * c] = (u32)wave_sum_i(nvalid[c]);
        v[2 * c + 1] = (u32)wave_sum_i(nkept[c]);
#pragma unroll
        for (int ww = 0; ww < 2; ++ww) {
            v[2 * kMaxC + 4 * c + 2 * ww] = f2ord(wave_minf(mn[c][ww]));
            v[2 * kMaxC + 4 * c + 2 * ww + 1] = f2ord(wave_maxf(mx[c][ww]));
        }
    }
    if (lane_id() == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) wred[w][k] = v[k];
    __syncthreads();
    if (t < NV) {
        const bool count = t < 2 * kMaxC;
        const int ws = t - 2 * kMaxC;                 // A_W offset of a statistic
        u32 r = wred[0][t];
        for (int ww = 1; ww < 4; ++ww) {
            const u32 o = wred[ww][t];
            if (count) r += o;
            else r = (ws & 1) ? max(r, o) : min(r, o);
        }
        if (count) {
            const int slot = (t & 1) ? C_KEPT + t / 2 : C_VALID + t / 2;
            if (r) atomicAdd(&a.cnt[slot], (int)r);
        } else if (ws & 1) {                                           // A_W + 4 c + 2 ww + 1: max
            if (r != f2ord(-FLT_MAX)) atomicMax(&a.acc[A_W + ws], r);
        } else if (r != f2ord(FLT_MAX)) {                              // A_W + 4 c + 2 ww: min
            atomicMin(&a.acc[A_W + ws], r);
        }
    }
}

// the p-index increments of an outer iteration: g = min(255, g + 1) once per valid query sharing the
// map point (:345-346, :493-496), applied by the last pair of each map point's list, which also
// empties the list for the next iteration
template <int NC>
__device__ __forceinline__ void pidx_apply(const int* nbr, const u32* tailinc, int n, const CatIdx<NC>& qi, CloudsW map,
                                           int4* pbkt, u32 map_cap) {
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const u32 inc = tailinc[p];
        if (!inc) continue;
        const int c = qi.cls(p / 5);
        float4* mp = map.at(c);
        const int idx = nbr[p];
        const float4 m = mp[idx];
        const u32 g = min(255u, w_g(m) + inc);
        mp[idx].w = __uint_as_float(pack_rg(w_r(m), g));
        int4* b = pbkt + (size_t)kBktQuads * ((u32)c * map_cap + (u32)idx);   // empty bucket
        b[0].x = 0;
        reinterpret_cast<int*>(b)[kBktHead] = -1;
    }
}

// the rgbds input of every class: its map, then its appended points (map c, app c, in class order)
template <int NC>
struct RgView {
    Clouds map, app;
    int m[kMaxC];          // map sizes
    int end[kMaxC];        // cumulative (map + appended) sizes
    __device__ __forceinline__ int total() const { return end[NC - 1]; }
    // class c, local index li, appended or not, of element v
    __device__ __forceinline__ void locate(int v, int& c, int& li, bool& appended) const {
        c = NC == 2 ? (v < end[0] ? 0 : 1) : (v < end[0] ? 0 : (v < end[1] ? 1 : 2));
        const int l = v - sel3(c, 0, end[0], end[1]);
        const int mc = sel3(c, m[0], m[1], m[2]);
        appended = l >= mc;
        li = appended ? l - mc : l;
    }
    __device__ __forceinline__ float4 at(int v, int& c) const {
        int li;
        bool ap;
        locate(v, c, li, ap);
        return (ap ? app.at(c) : map.at(c))[li];
    }
};

template <int NC>
__device__ __forceinline__ RgView<NC> rg_view(const int* cnt, Clouds map, Clouds app) {
    RgView<NC> V;
    V.map = map;
    V.app = app;
    int acc = 0;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
        V.m[c] = c < NC ? cnt[C_M + c] : 0;
        acc += c < NC ? cnt[C_M + c] + cnt[C_DS + c] : 0;
        V.end[c] = acc;
    }
    return V;
}

constexpr int kRgmThreads = 256;
constexpr int kRgmBuckets = 512;
constexpr int kRgmBucketCap = 2048;     // appended points a bucket sorts
constexpr int kRgmOldLds = 1024;        // map points (keys, points) of a bucket cached in LDS
constexpr int kRgmAppLds = 512;         // appended points of a bucket cached in LDS (sorted order)
constexpr u32 kRgmDrop = 0x80000000u;

// the frame's crop box (as k_rg_append_keys)
struct RgmBox {
    float lo[3], hi[3];
    __device__ __forceinline__ bool in(float4 p) const {
        return !((p.x < lo[0] || p.y < lo[1] || p.z < lo[2]) || (p.x > hi[0] || p.y > hi[1] || p.z > hi[2]));
    }
};
__device__ __forceinline__ RgmBox rgm_box(const double* prm) {
    RgmBox b;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        b.lo[k] = (float)(prm[4 + k] - 100);
        b.hi[k] = (float)(prm[4 + k] + 100);
    }
    return b;
}
// voxel coordinate floor(v / lf) relative to the crop box's voxel origin, biased by 2^19 and clamped
// (monotone, so the order of clamped keys is the order of the points; inside the box exact)
__device__ __forceinline__ u64 rgm_axis(float v, float lo, float lf) {
    float d = floorf(v / lf) - (float)(int)floorf(lo / lf);
    d = fminf(fmaxf(d, -524288.f), 524287.f);
    return (u64)((int)d + 524288);
}
__device__ __forceinline__ u64 rgm_key(float4 p, int c, float lf, const RgmBox& b) {
    return ((u64)c << 62) | (rgm_axis(p.z, b.lo[2], lf) << 40) | (rgm_axis(p.y, b.lo[1], lf) << 20) |
           rgm_axis(p.x, b.lo[0], lf);
}
__device__ __forceinline__ bool rgm_less(u64 ka, u32 ta, u64 kb, u32 tb) {
    return ka < kb || (ka == kb && (ta & ~kRgmDrop) < (tb & ~kRgmDrop));
}

// element index of map point g (map order over the classes) / appended point a
template <int NC>
__device__ __forceinline__ int rgm_old_elem(const RgView<NC>& V, int g, int& c, int& li) {
    int start = 0, acc = 0;
    c = NC - 1;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        const int mk = V.m[k];
        if (g < acc + mk) { c = k; break; }
        acc += mk;
        start = V.end[k];
    }
    li = g - acc;
    return start + li;
}
template <int NC>
__device__ __forceinline__ int rgm_app_elem(const RgView<NC>& V, int a, int& c, int& li) {
    int start = 0, acc = 0;
    c = NC - 1;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        const int ak = V.end[k] - (k ? V.end[k - 1] : 0) - V.m[k];
        if (a < acc + ak) { c = k; break; }
        acc += ak;
        start = V.end[k];
    }
    li = a - acc;
    const int mc = sel3(c, V.m[0], V.m[1], V.m[2]);
    return start + mc + li;
}
template <int NC>
__device__ __forceinline__ float4 rgm_old_point(const RgView<NC>& V, int g, int& c) {
    int li;
    (void)rgm_old_elem<NC>(V, g, c, li);
    return V.map.at(c)[li];
}
template <int NC>
__device__ __forceinline__ u64 rgm_old_key(const RgView<NC>& V, const VgLeaf& leaf, const RgmBox& box, int g) {
    int c;
    const float4 p = rgm_old_point<NC>(V, g, c);
    return rgm_key(p, c, leaf.at(c), box);
}

// First map element (classes concatenated) of bucket b; bucket b merges map elements
// [rgm_bucket_lo(b), rgm_bucket_lo(b + 1)). Every class with map points gets at least
// ceil(2 a_c / kRgmBucketCap) buckets, so its appended points average at most half a list even when
// its map is small next to another class's (configs[4]: a 7k-point edge map beside a 2M-point surf
// map); the remaining buckets go by map size, and a class's map range is split evenly.
template <int NC>
__device__ __forceinline__ int rgm_bucket_lo(const RgView<NC>& V, int b) {
    int M = 0, need = 0, want[kMaxC] = {0, 0, 0};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int a = V.end[c] - (c ? V.end[c - 1] : 0) - V.m[c];
        want[c] = V.m[c] > 0 ? max(1, (2 * a + kRgmBucketCap - 1) / kRgmBucketCap) : 0;
        need += want[c];
        M += V.m[c];
    }
    if (M == 0) return 0;
    if (need > kRgmBuckets) return (int)(((long long)b * M) / kRgmBuckets);   // the plain split
    const int rem = kRgmBuckets - need;
    int nb[kMaxC] = {0, 0, 0}, given = 0, last = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        nb[c] = want[c] + (int)(((long long)rem * V.m[c]) / M);
        given += nb[c];
        if (V.m[c] > 0) last = c;
    }
    nb[last] += kRgmBuckets - given;
    int b0 = 0, m0 = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (nb[c] > 0 && b < b0 + nb[c]) return m0 + (int)(((long long)(b - b0) * V.m[c]) / nb[c]);
        b0 += nb[c];
        m0 += V.m[c];
    }
    return M;
}

// lower / upper bound of k in sorted keys[0 .. n) (LDS or global)
__device__ __forceinline__ int rgm_lower(const u64* keys, int n, u64 k) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int rgm_upper(const u64* keys, int n, u64 k) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] <= k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The rgbds merge's appended points, prepared by the last LM launch of an update (k_lm_solve's
// workgroups, once the pose is solved): pointAssociateToMap (:592-604) of every down-sampled point
// with the solved parameters x, its voxel key and crop flag, and its bucket (k_rgm_bucket): every
// workgroup takes the buckets' splitters (the keys of map points b M / R) into LDS, and each point is
// appended to its bucket's list (unordered; the bucket sorts it) with one counter atomic. A list
// past kRgmBucketCap points sets the fallback flag.
struct RgmPrep {
    int on;
    Clouds map, ds;
    CloudsW app;
    u64* key64;
    u32* vtag;
    VgLeaf leaf;
    u32* bcount;           // [kRgmBuckets] list sizes (each zeroed by k_rgm_finish after its bucket is merged)
    u64* bkey;             // [kRgmBuckets][kRgmBucketCap]
    u32* btag;
    int* stat;             // rgm_stat: [0] fallback flag
};
template <int NC>
__device__ void rgm_prep_apps(const RgmPrep& r, const int* cnt, const double* x) {
    __shared__ u64 s_sp[kRgmBuckets];
    const RgView<NC> V = rg_view<NC>(cnt, r.map, Clouds{{nullptr, nullptr, nullptr}});
    int M = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) M += V.m[c];
    const int A = V.total() - M;
    double prm[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) prm[k] = x[k];
    const RgmBox box = rgm_box(prm);
    for (int i = threadIdx.x; i < kRgmBuckets; i += blockDim.x) {
        const int l0 = rgm_bucket_lo<NC>(V, i);
        s_sp[i] = i == 0 ? 0ull : (l0 >= M ? ~0ull : rgm_old_key<NC>(V, r.leaf, box, l0));
    }
    __syncthreads();
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < A; q += gridDim.x * blockDim.x) {
        int c, li;
        const int e = rgm_app_elem<NC>(V, q, c, li);
        float4 p = r.ds.at(c)[li];
        p.w = __uint_as_float(__hip_atomic_load(reinterpret_cast<const u32*>(&r.ds.at(c)[li].w), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));   // r / g: the fused observe pass
        p = associate(prm, p);
        r.app.at(c)[li] = p;
        const u64 key = rgm_key(p, c, r.leaf.at(c), box);
        const u32 tag = (u32)e | (box.in(p) ? 0u : kRgmDrop);
        r.key64[e] = key;
        r.vtag[e] = tag;
        int o = 0;                                    // largest bucket whose splitter is <= key
#pragma unroll
        for (int step = kRgmBuckets / 2; step > 0; step >>= 1)
            if (s_sp[o + step] <= key) o += step;
        const u32 slot = atomicAdd(&r.bcount[o], 1u);
        if (slot < (u32)kRgmBucketCap) {
            r.bkey[(size_t)o * kRgmBucketCap + slot] = key;
            r.btag[(size_t)o * kRgmBucketCap + slot] = tag;
        } else {
            r.stat[0] = 1;
        }
    }
}

// ------------------------------------ LM (B.6) ----------------------------------------------
// Ceres 1.14 trust-region loop of one outer iteration in ONE launch. Per evaluation (<= 1 + kMaxIter
// = 5) the kept residual blocks are split into kLmBlocks fixed *chunks* (chunk c = the queries
// c * 256 + k * kLmBlocks * 256, k = 0, 1, ...); workgroup b reduces its home chunk b to 30 partials
// (cost, g, upper J^T J, bad counts) and stores them write-through over sentinel values, so each
// partial is its own completion flag. Once no partial of the evaluation is a sentinel any more,
// every workgroup combines the partials in chunk order and takes the LM step itself
// (TrustRegionMinimizer + LevenbergMarquardtStrategy): the step is a deterministic function of
// identical inputs, so every workgroup holds the same LM state and nothing is broadcast.
// Forward progress does not depend on co-residency: chunks are claimed on a per-evaluation mask, a
// waiting workgroup claims and reduces the chunks nobody has claimed (home workgroups not started),
// and one that starts late finds its chunk claimed and replays the steps from the stored partials. So any number of solves may be in flight
// on a device. The reduction tree (chunk partials summed in chunk order) is independent of which
// workgroup ran which chunk, so the result is bit-identical however the chunks were dealt out.
// A wait that exceeds its bound (a bug, never expected) sets C_ERR and the sticky error word.
constexpr unsigned kLmStealPolls = 64;      // polls (~1 us each) before a waiting block steals chunks

// observeMean (:136-160) / pointSparsityMean (.h:111-126) of one element, given min/max
__device__ __forceinline__ double norm_weight(double e, double mn, double mx, bool clamp) {
    const double length = mx - mn;
    if (length == 0) return e;
    e = (e - mn) / length;
    e -= 1.0;
    e = fabs(e);
    e *= 2.0;
    if (clamp) e = fmax(0.1, e);
    return e;
}

// packed symmetric 6x6: lm->H holds the upper triangle row by row (i <= j)
__device__ __forceinline__ int hup(int i, int j) {
    if (i > j) { const int t = i; i = j; j = t; }
    return i * 6 - (i * (i - 1)) / 2 + (j - i);
}
__device__ __forceinline__ int tri(int i, int j) { return i * (i + 1) / 2 + j; }   // lower, j <= i

// The LM state lanes 0 and 1 work on during a step: x, cand and the scalars in registers (loaded
// from / stored to the LDS LMState around it); scale, g, H and D are read and written in place in
// the LDS LMState (both lanes write identical values), so the step's live set fits the 256
// architected VGPRs (held in registers, the 6x6 state spilled into AGPR moves: a third of the
// step's instructions). Every loop is fully unrolled so all indices are static.
struct LmCore {
    double x[7], cand[7];
    double *scale, *g, *H, *D;                                   // -> LMState (LDS)
    double cost, radius, decrease, x_norm, min_cost, mcc;
    int iteration, invalid, reuse, done, phase;
};
__device__ __forceinline__ void core_load(LmCore& c, LMState& s) {
    c.scale = s.scale;
    c.g = s.g;
    c.H = s.H;
    c.D = s.D;
#pragma unroll
    for (int k = 0; k < 7; ++k) { c.x[k] = s.x[k]; c.cand[k] = s.cand[k]; }
    c.cost = s.cost; c.radius = s.radius; c.decrease = s.decrease; c.x_norm = s.x_norm;
    c.min_cost = s.min_cost; c.mcc = s.mcc;
    c.iteration = s.iteration; c.invalid = s.invalid; c.reuse = s.reuse; c.done = s.done; c.phase = s.phase;
}
__device__ __forceinline__ void core_store(const LmCore& c, LMState& s) {
#pragma unroll
    for (int k = 0; k < 7; ++k) { s.x[k] = c.x[k]; s.cand[k] = c.cand[k]; }
    s.cost = c.cost; s.radius = c.radius; s.decrease = c.decrease; s.x_norm = c.x_norm;
    s.min_cost = c.min_cost; s.mcc = c.mcc;
    s.iteration = c.iteration; s.invalid = c.invalid; s.reuse = c.reuse; s.done = c.done; s.phase = c.phase;
}

// One attempt of LevenbergMarquardtStrategy::ComputeStep on the current state, without mutating it:
// D (fresh from diag(Hs) unless reused), the LDL^T factorisation of Hs + D / radius (no square
// roots; one reciprocal per pivot, multiplied in: 6 divisions on the serial chain instead of the
// 27 of a Cholesky with divided substitutions), the step y (delta = -y .* scale) and the model cost
// change mcc. Every multiply-subtract of the factorisation, the two solves and the mcc sums is one
// explicit fused multiply-add (one rounding; the oracle's GPU_EQUIV restates it with std::fma), which
// halves the dependent chain of the serial step. Hs entries are recomputed from H. A pivot <= 0 rejects the step, as a Cholesky's
// non-positive square-root argument does (both test positive definiteness).
struct StepTry {
    double y[6], D[6], mcc;
    bool ok;
};
__device__ __forceinline__ StepTry lm_try_step(const LmCore& lm) {
    StepTry r;
#pragma unroll
    for (int j = 0; j < 6; ++j)
        r.D[j] = lm.reuse ? lm.D[j] : fmin(fmax(lm.scale[j] * lm.H[hup(j, j)] * lm.scale[j], 1e-6), 1e32);
    double A[21];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) A[tri(i, j)] = lm.scale[i] * lm.H[hup(i, j)] * lm.scale[j];
    const double ir = 1.0 / lm.radius;
#pragma unroll
    for (int j = 0; j < 6; ++j) A[tri(j, j)] += r.D[j] * ir;
    // LDL^T in place: A[tri(i, j)] (j < i) becomes L_ij, W holds L_ij d_j, inv[j] = 1 / d_j
    double W[21], inv[6];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
#pragma unroll
        for (int j = 0; j < i; ++j) {
            double s = A[tri(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) s = fma(-W[tri(i, k)], A[tri(j, k)], s);
            W[tri(i, j)] = s;
            A[tri(i, j)] = s * inv[j];
        }
        double d = A[tri(i, i)];
#pragma unroll
        for (int k = 0; k < i; ++k) d = fma(-W[tri(i, k)], A[tri(i, k)], d);
        ok = ok && (d > 0.0);
        inv[i] = 1.0 / d;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {                                // L z = scale .* g
        double s = lm.scale[i] * lm.g[i];
#pragma unroll
        for (int k = 0; k < i; ++k) s = fma(-A[tri(i, k)], r.y[k], s);
        r.y[i] = s;
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {                               // L^T y = D^-1 z
        double s = r.y[i] * inv[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) s = fma(-A[tri(k, i)], r.y[k], s);
        r.y[i] = s;
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) ok = ok && isfinite(r.y[j]);
    r.mcc = 0.0;
    if (ok) {
        double sg = 0.0, sHs = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            sg = fma(-r.y[i], lm.scale[i] * lm.g[i], sg);
            double hi = 0.0;
#pragma unroll
            for (int j = 0; j < 6; ++j) hi = fma(lm.scale[i] * lm.H[hup(i, j)] * lm.scale[j], -r.y[j], hi);
            sHs = fma(-r.y[i], hi, sHs);
        }
        r.mcc = -(sg + 0.5 * sHs);
    }
    r.ok = ok && (r.mcc > 0.0);
    return r;
}

// TrustRegionMinimizer + LevenbergMarquardtStrategy: next candidate, or done (the retry loop of
// invalid steps; its first attempt `first` has already been computed)
__device__ __forceinline__ void lm_next_step(LmCore& lm, StepTry st, const double* cand_first) {
    const int kMaxIter = 4;
    for (bool first = true;; first = false) {
        lm.iteration++;
        if (!first) st = lm_try_step(lm);
        if (!lm.reuse) {
#pragma unroll
            for (int j = 0; j < 6; ++j) lm.D[j] = st.D[j];
        }
        lm.reuse = 1;
        if (!st.ok) {                                    // invalid step (HandleInvalidStep)
            if (++lm.invalid >= 5) { lm.done = 1; return; }
            lm.radius = lm.radius / lm.decrease;
            lm.decrease *= 2.0;
            if (lm.iteration >= kMaxIter || lm.radius <= 1e-32) { lm.done = 1; return; }
            continue;
        }
        lm.invalid = 0;
        if (first) {
#pragma unroll
            for (int k = 0; k < 7; ++k) lm.cand[k] = cand_first[k];
        } else {
            double delta[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) delta[j] = -st.y[j] * lm.scale[j];
            se3_plus(lm.x, delta, lm.cand);
        }
        lm.mcc = st.mcc;
        lm.phase = 1;
        return;
    }
}

// Evaluation `tot` (cost, g, H, bad_r, bad_J) of lm.cand -> update the LM state. Run by lanes 0 and
// 1 of a wave on identical state: the gradient-norm check x (+) (-g) and the next candidate
// x (+) delta are the same SE(3) update, so lane 0 evaluates the first and lane 1 the second at
// once (the candidate is computed speculatively and discarded when the check ends the solve).
// best: the LDS copy (LMState::best), written by both lanes with identical values
__device__ __forceinline__ void lm_accept(LmCore& lm, const double* tot, double* best, unsigned long long* pr = nullptr) {
    const double cost_c = tot[0];
    const bool bad_r = tot[28] > 0.0, bad_j = tot[29] > 0.0;
    const int kMaxIter = 4;
    bool step_ok = false;
    if (lm.phase == 0) {                                         // IterationZero
        if (bad_r || bad_j) {
            lm.done = 1;
            return;
        }
        lm.cost = cost_c;
#pragma unroll
        for (int k = 0; k < 6; ++k) lm.g[k] = tot[1 + k];
#pragma unroll
        for (int k = 0; k < 21; ++k) lm.H[k] = tot[7 + k];
#pragma unroll
        for (int i = 0; i < 6; ++i) lm.scale[i] = 1.0 / (1.0 + sqrt(lm.H[hup(i, i)]));   // Jacobi, once
        lm.min_cost = lm.cost;
#pragma unroll
        for (int k = 0; k < 7; ++k) best[k] = lm.x[k];
        step_ok = true;                                          // gradient check below
    } else {
        const double cand_cost = bad_r ? DBL_MAX : cost_c;       // candidate evaluated
        double sn = 0.0;
#pragma unroll
        for (int j = 0; j < 7; ++j) sn += (lm.x[j] - lm.cand[j]) * (lm.x[j] - lm.cand[j]);
        sn = sqrt(sn);
        if (sn <= 1e-8 * (lm.x_norm + 1e-8)) {
            lm.done = 1;                                         // parameter tolerance
            return;
        }
        if (fabs(lm.cost - cand_cost) <= 1e-6 * lm.cost) {
            lm.done = 1;                                         // function tolerance
            return;
        }
        const double rel = (lm.cost - cand_cost) / lm.mcc;
        if (rel > 1e-3) {
            double xn = 0;
#pragma unroll
            for (int j = 0; j < 7; ++j) { lm.x[j] = lm.cand[j]; xn += lm.x[j] * lm.x[j]; }
            lm.x_norm = sqrt(xn);
            if (bad_j) {
                lm.done = 1;                                     // Jacobian evaluation failed
                return;
            }
            lm.cost = cand_cost;
#pragma unroll
            for (int k = 0; k < 6; ++k) lm.g[k] = tot[1 + k];
#pragma unroll
            for (int k = 0; k < 21; ++k) lm.H[k] = tot[7 + k];
            const double r3 = 2.0 * rel - 1.0;
            const double f = 1.0 - r3 * r3 * r3;                 // std::pow(2 rel - 1, 3)
            lm.radius = lm.radius / fmax(1.0 / 3.0, f);
            lm.radius = fmin(1e16, lm.radius);
            lm.decrease = 2.0;
            lm.reuse = 0;
            step_ok = true;
            if (lm.cost < lm.min_cost) {
                lm.min_cost = lm.cost;
#pragma unroll
                for (int k = 0; k < 7; ++k) best[k] = lm.x[k];
            }
        } else {
            lm.radius = lm.radius / lm.decrease;
            lm.decrease *= 2.0;
            lm.reuse = 1;
        }
        if (lm.iteration >= kMaxIter) {
            lm.done = 1;
            return;
        }
    }
    // the first attempt of the next step, and both SE(3) updates on two lanes
    if (pr) pr[0] = __builtin_amdgcn_s_memrealtime();
    const StepTry st = lm_try_step(lm);
    if (pr) pr[1] = __builtin_amdgcn_s_memrealtime();
    const bool lane1 = (threadIdx.x & 1) != 0;
    double in[6], out[7];
#pragma unroll
    for (int j = 0; j < 6; ++j) in[j] = lane1 ? -st.y[j] * lm.scale[j] : -lm.g[j];
    se3_plus(lm.x, in, out);
    double cand[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) cand[k] = __shfl(out[k], (threadIdx.x & ~1) | 1, 64);
    double gm = 0.0;
#pragma unroll
    for (int j = 0; j < 7; ++j) gm = fmax(gm, fabs(lm.x[j] - out[j]));
    gm = __shfl(gm, threadIdx.x & ~1, 64);                       // lane 0's gradient max-norm
    if (pr) pr[2] = __builtin_amdgcn_s_memrealtime();
    if (step_ok && gm <= 1e-10) lm.done = 1;
    else if (lm.phase != 0 && lm.radius <= 1e-32) lm.done = 1;
    else lm_next_step(lm, st, cand);
}

// the inputs of one residual block as the evaluation reads them
struct ResIn {
    d3 cur;
    double G[6];
    double wgt;
    bool kept, plane;
};

struct LmArgs {
    DevState* st;
    int* cnt;
    const u32* acc;
    ClassCfg cls;
    LMState* lm_out;
    double* part;          // [kLmEvals][kLmBlocks][32]
    u32* arrive;           // arrival counter, zeroed by k_assoc
    const int* qflag;
    Clouds ds;
    const double* geo;
    const float* observe;
    const float* spars;
    int weight_type;
    unsigned long long* dbg;
    const int* nbr;        // p-index increments, applied by the LM blocks before the solve
    const u32* tailinc;
    int4* pbkt;
    CloudsW map;
    u32 map_cap;
    int* err;              // sticky error word E_LM
    RgmPrep prep;          // the last launch of an update prepares the rgbds merge's appended points
    ObsArgs obs;           // fuse: the observe pass runs here, chunk by chunk (weightType 0; k_observe not launched)
    int fuse;
};

// one pair's p-index increment (pidx_apply's body)
__device__ __forceinline__ void pidx_apply_pair(const int* nbr, u32 inc, int p, int c, CloudsW map, int4* pbkt,
                                                u32 map_cap) {
    float4* mp = map.at(c);
    const int idx = nbr[p];
    const float4 m = mp[idx];
    const u32 g = min(255u, w_g(m) + inc);
    mp[idx].w = __uint_as_float(pack_rg(w_r(m), g));
    int4* b = pbkt + (size_t)kBktQuads * ((u32)c * map_cap + (u32)idx);   // empty bucket
    b[0].x = 0;
    reinterpret_cast<int*>(b)[kBktHead] = -1;
}

// the p-index increments of the chunks in mask m (k_lm_solve's fused observe pass), by threads i0,
// i0 + ni, ... of the workgroup; out of line, so the solve's register allocation does not carry it
template <int NC>
__device__ __noinline__ void lm_apply_commits(const int* nbr, const u32* tailinc, CloudsW map, int4* pbkt, u32 map_cap,
                                              CatIdx<NC> qi, int nq, u32 m, int i0, int ni) {
    for (int ch = 0; ch < kLmBlocks; ++ch) {
        if (!((m >> ch) & 1u)) continue;
        for (int base = ch * 256; base < nq; base += kLmBlocks * 256)
            for (int i = i0; i < 256; i += ni) {
                const int q = base + i;
                if (q >= nq) continue;
                const int c = qi.cls(q);
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const u32 inc = tailinc[5 * q + j];
                    if (inc) pidx_apply_pair(nbr, inc, 5 * q + j, c, map, pbkt, map_cap);
                }
            }
    }
}

template <int NC>
__global__ void __launch_bounds__(256) k_lm_solve(LmArgs a) {
    unsigned long long* dbg = a.dbg;
    const bool rec = dbg && blockIdx.x == 0 && threadIdx.x == 0;
    if (rec) dbg[0] = __builtin_amdgcn_s_memrealtime();
    // per-workgroup probe (every block's thread 0): start, and per evaluation the home chunk's
    // publish and the end of the arrival wait
    unsigned long long* recb = dbg && threadIdx.x == 0 ? dbg + kLmBlkProbe : nullptr;
    if (recb) recb[2 * kLmEvals * kLmBlocks + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    __shared__ double rows[256][9];                             // per residual: J[6], r, 0.5 rho (+1 pad:
                                                                // a stride of 18 words spreads a wave's rows over the 32 banks)
    __shared__ double red9[28][9];
    __shared__ int nbad[3];                                     // bad residuals, bad Jacobians, kept rows
    __shared__ double tot[kLmParts];
    __shared__ LMState lm;
    __shared__ int aborted;
    const int t = threadIdx.x;
    // the map's p-index bytes are not read by the solve: this iteration's increments are applied while
    // the blocks wait for the first evaluation's arrivals (k_observe launched), beside the first LM step
    // (observe pass fused), or here when there is no solve.
    // Every value the set-up reads from memory is loaded here, in one round trip: the counts, the gate
    // and (thread 0) the pose
    const CatIdx<NC> qi = cat_idx<NC>(a.cnt + C_DS);
    const int nq = a.cnt[C_NQ];
    const int gate = a.st->gate;
    double prm0[7];
    if (t == 0)
        for (int k = 0; k < 7; ++k) prm0[k] = a.st->params[k];
    // fused observe pass (weightType 0): the residual count is known after the first evaluation
    // (its partials carry each chunk's kept rows); without a gate there is nothing to observe
    const bool fuse = a.fuse != 0;
    int nres = 0;
    if (!fuse)
        for (int c = 0; c < NC; ++c) nres += a.cnt[C_KEPT + c];
    if (!gate || (!fuse && nres == 0)) {                         // no residual blocks: untouched
        if (!fuse) pidx_apply(a.nbr, a.tailinc, a.cnt[C_NPAIR], qi, a.map, a.pbkt, a.map_cap);
        if (a.prep.on) rgm_prep_apps<NC>(a.prep, a.cnt, a.st->params);
        return;
    }
    // the weight bounds and this thread's home residual live in LDS, not in registers: the serial
    // LM step of lanes 0 / 1 needs the register file (long-lived values spill it to AGPR moves)
    __shared__ double wmin[kMaxC][2], wmax[kMaxC][2];
    __shared__ ResIn s_mine[256];
    if (t < 2 * kMaxC) {
        const int c = t >> 1, ww = t & 1;
        wmin[c][ww] = (double)ord2f(a.acc[A_W + 4 * c + 2 * ww]);
        wmax[c][ww] = (double)ord2f(a.acc[A_W + 4 * c + 2 * ww + 1]);
    }
    if (t == 0) {                                                // problem set-up (:252-266)
        double xn = 0;
        for (int k = 0; k < 7; ++k) {
            lm.x[k] = lm.cand[k] = lm.best[k] = prm0[k];
            xn += prm0[k] * prm0[k];
        }
        lm.x_norm = sqrt(xn);
        lm.radius = 1e4;
        lm.decrease = 2.0;
        lm.iteration = lm.invalid = lm.reuse = lm.phase = 0;
        lm.n_res = nres;
        lm.done = 0;
        aborted = 0;
        nbad[0] = nbad[1] = nbad[2] = 0;                         // before the barrier: every wave may count
    }
    __syncthreads();
    const int wt = a.weight_type;
    // reduction roles: thread (k, p) sums product k (0: cost, 1-6: g, 7-27: upper J^T J, row by row)
    // over the chunk rows p, p + 9, ...; 28 x 9 = 252 threads
    const int rk = t / 9, rp = t % 9;
    int ri = 0, rj_ = 0;
    if (rk >= 7 && rk < 28) {
        int h = rk - 7;
        while (h >= 6 - ri) { h -= 6 - ri; ++ri; }
        rj_ = ri + h;
    }
    // chunk c of an evaluation = the queries c * 256 + k * kLmBlocks * 256; block b first reduces its
    // home chunk b and claims it with one atomicOr on the evaluation's claim mask, whose result is
    // only needed when the partials are published (the atomic's latency hides behind the reduction).
    // A block waiting for the evaluation to complete claims unclaimed chunks after kLmStealPolls
    // polls: only chunks of workgroups that have not started yet stay unclaimed that long.
    static_assert(kLmBlocks <= 32, "one claim-mask word per evaluation");
    constexpr u32 kFull = (u32)((1ull << kLmBlocks) - 1ull);
    __shared__ int s_won, s_state, s_steal;
    u32* claim = a.arrive;                                       // [kLmEvalSlots] claim masks
    double x[7];
    // one residual's inputs: the down-sampled point, the line (a, b) or plane (n, d) and the weight
    // (fused: the kept bit may come from another workgroup of this launch, written through)
    auto load_flag = [&](int q) {
        return fuse ? __hip_atomic_load(&a.qflag[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : a.qflag[q];
    };
    auto load_res_k = [&](int q, bool kept) {
        ResIn in{};
        if (kept) {
            in.kept = true;
            const int c = qi.cls(q);
            in.plane = c == NC - 1;                              // the last class is the plane class
            const float4 p = a.ds.at(c)[q - qi.start(c)];
            in.cur = d3{(double)p.x, (double)p.y, (double)p.z};
            if (wt != 0) {
                const double wo = norm_weight((double)a.observe[q], sel3(c, wmin[0][0], wmin[1][0], wmin[2][0]),
                                              sel3(c, wmax[0][0], wmax[1][0], wmax[2][0]), true);
                const double ws = norm_weight((double)a.spars[q], sel3(c, wmin[0][1], wmin[1][1], wmin[2][1]),
                                              sel3(c, wmax[0][1], wmax[1][1], wmax[2][1]), false);
                if (wt == 1) in.wgt = wo;
                else if (wt == 2) in.wgt = ws;
                else in.wgt = in.plane ? (wo + ws) / 2 : (ws + wo) / 2;     // :418 / :565 operand order
            }
            const double* G = a.geo + 8 * (size_t)q;
            for (int k = 0; k < 6; ++k) in.G[k] = G[k];
        }
        return in;
    };
    auto load_res = [&](int q) { return load_res_k(q, q < nq && (load_flag(q) & 2)); };
    // the observe pass of chunk ch (fused): every slice's queries evaluated, their outputs committed
    // when this workgroup owns the chunk's first evaluation (won), the valid / kept counts added
    __shared__ u32 s_commit, s_claim0;
    __shared__ int s_ocnt[2 * kMaxC];
    auto observe_chunk = [&](int ch, bool home_claim) -> bool {
        if (rec && home_claim) dbg[55] = __builtin_amdgcn_s_memrealtime();
        if (t < 2 * kMaxC) s_ocnt[t] = 0;
        bool kept0 = false, won = true;
        for (int base = ch * 256, k = 0; base < nq; base += kLmBlocks * 256, ++k) {
            const int q = base + t;
            ObsRes r;
            r.f = 0;
            if (q < nq) observe_eval<NC>(a.obs, qi, nq, q, r);
            if (rec && home_claim && k == 0) dbg[50] = __builtin_amdgcn_s_memrealtime();
            if (k == 0) {
                __syncthreads();                                 // s_claim0 (thread 0's claim) and s_ocnt
                if (rec && home_claim) dbg[51] = __builtin_amdgcn_s_memrealtime();
                won = !home_claim || ((s_claim0 >> ch) & 1u) == 0u;
                kept0 = (r.f & 1) && !r.skip;
            }
            if (won && q < nq) {
                observe_commit<NC>(a.obs, qi, q, r, true);
                if (r.f & 1) {
                    atomicAdd(&s_ocnt[2 * r.c], 1);
                    if (!r.skip) atomicAdd(&s_ocnt[2 * r.c + 1], 1);
                }
            }
        }
        // the commits complete before this chunk's partials are published (consumers that see the
        // partials read the kept bits)
        if (rec && home_claim) dbg[52] = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (rec && home_claim) dbg[53] = __builtin_amdgcn_s_memrealtime();
        if (won && t < 2 * NC && s_ocnt[t]) atomicAdd(&a.cnt[(t & 1) ? C_KEPT + t / 2 : C_VALID + t / 2], s_ocnt[t]);
        if (won && t == 0) s_commit |= 1u << ch;
        return kept0;
    };
    // the p-index increments of the chunks this workgroup observed, by threads i0, i0 + ni, ... of the
    // workgroup (after the first evaluation's arrivals: every observe pass of the launch has read the
    // map's g bytes)
    auto apply_commits = [&](int i0, int ni) {
        lm_apply_commits<NC>(a.nbr, a.tailinc, a.map, a.pbkt, a.map_cap, qi, nq, s_commit, i0, ni);
    };
    u32 old0 = 0;
    bool applied = !fuse;
    if (fuse) {
        if (t == 0) {
            s_commit = 0u;
            s_claim0 = __hip_atomic_fetch_or(&claim[0], 1u << blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const bool kept0 = observe_chunk((int)blockIdx.x, true);
        old0 = s_claim0;
        s_mine[t] = load_res_k((int)blockIdx.x * 256 + t, kept0);
        if (rec) dbg[54] = __builtin_amdgcn_s_memrealtime();
    } else {
        s_mine[t] = load_res((int)blockIdx.x * 256 + t);
    }
    // reduce chunk ch of evaluation ev at x into 30 partials; publish them and count the chunk done
    // unless another block claimed it first (own_claim: claim_old is this block's atomicOr result)
    auto reduce_chunk = [&](int ch, int ev, u32 claim_old, bool own_claim) {
        double part = 0.0;
        for (int base = ch * 256; base < nq; base += kLmBlocks * 256) {
            const int q = base + t;
            double J[6] = {0, 0, 0, 0, 0, 0}, r = 0.0, hc = 0.0;
            // the inputs of this thread's residual: from registers for the home chunk's first rows
            // (`s_mine`, loaded once per launch), from memory otherwise
            const bool cached = ch == (int)blockIdx.x && base == ch * 256;
            const ResIn in = cached ? s_mine[t] : load_res(q);
            if (in.kept) {
                atomicAdd(&nbad[2], 1);
                r = in.plane ? surf_eval(x, in.cur, d3{in.G[0], in.G[1], in.G[2]}, in.G[3], in.wgt, J)
                             : edge_eval(x, in.cur, d3{in.G[0], in.G[1], in.G[2]}, d3{in.G[3], in.G[4], in.G[5]},
                                         in.wgt, J);
                bool jbad = false;
                for (int k = 0; k < 6; ++k) jbad |= !isfinite(J[k]);
                if (!isfinite(r)) {
                    atomicAdd(&nbad[0], 1);
                    r = 0.0;
                    for (int k = 0; k < 6; ++k) J[k] = 0.0;
                } else {
                    if (jbad) atomicAdd(&nbad[1], 1);
                    const double s = r * r;                      // HuberLoss(0.1) + Corrector
                    double rho0, rho1;
                    if (s > 0.1 * 0.1) {
                        const double rr = sqrt(s);
                        rho0 = 2.0 * 0.1 * rr - 0.1 * 0.1;
                        rho1 = fmax(DBL_MIN, 0.1 / rr);
                    } else {
                        rho0 = s;
                        rho1 = 1.0;
                    }
                    hc = 0.5 * rho0;
                    const double sr = sqrt(rho1);
                    r *= sr;
                    for (int k = 0; k < 6; ++k) J[k] *= sr;
                }
            }
            for (int k = 0; k < 6; ++k) rows[t][k] = J[k];
            rows[t][6] = r;
            rows[t][7] = hc;
            __syncthreads();
            if (rk < 28) {                                       // rows rp*29 .. rp*29+28
                const int ca = rk == 0 ? 7 : (rk < 7 ? rk - 1 : ri), cb = rk == 0 ? -1 : (rk < 7 ? 6 : rj_);
                // in groups of 8 rows: every group's LDS reads issued at once, the sum in row order
#pragma unroll
                for (int i0 = 0; i0 < 29; i0 += 8) {
                    double pa[8], pb[8];
#pragma unroll
                    for (int i = 0; i < 8 && i0 + i < 29; ++i) {
                        const int j = rp * 29 + i0 + i;
                        pa[i] = j < 256 ? rows[j][ca] : 0.0;
                        pb[i] = (j < 256 && cb >= 0) ? rows[j][cb] : 1.0;
                    }
#pragma unroll
                    for (int i = 0; i < 8 && i0 + i < 29; ++i) part += pa[i] * pb[i];
                }
            }
            __syncthreads();
        }
        if (rk < 28) red9[rk][rp] = part;
        if (t == 0) s_won = own_claim ? ((claim_old >> ch) & 1u) == 0u : 1;
        __syncthreads();
        // publish: write-through (agent-scope atomic) stores of the 30 partials over the sentinels
        // k_assoc left there; each value is its own completion flag, so nothing waits for the stores
        // and no counter is bumped (consumers poll the values with agent-scope atomic loads)
        double* P = a.part + (size_t)ev * kLmBlocks * 32;
        const bool pub = s_won != 0;
        if (t < 28) {
            double v = red9[t][0];
            for (int k = 1; k < 9; ++k) v += red9[t][k];
            if (pub) __hip_atomic_store(P + 32 * ch + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (t < kLmParts) {
            if (pub) __hip_atomic_store(P + 32 * ch + t, (double)nbad[t - 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nbad[t - 28] = 0;                                    // for the next chunk (after the barrier)
        }
        __syncthreads();
    };
    for (int ev = 0; ev < kLmEvals; ++ev) {
        if (lm.done || aborted) break;                           // uniform: every block steps alike
        for (int k = 0; k < 7; ++k) x[k] = lm.cand[k];
        const int home = blockIdx.x;                             // grid == kLmBlocks
        u32 old = 0;
        if (fuse && ev == 0) old = old0;                         // claimed before the observe pass
        else if (t == 0) old = __hip_atomic_fetch_or(&claim[ev], 1u << home, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        reduce_chunk(home, ev, old, true);
        if (rec) dbg[1 + 4 * ev] = dbg[2 + 4 * ev] = __builtin_amdgcn_s_memrealtime();
        if (recb) recb[2 * (ev * kLmBlocks + home)] = __builtin_amdgcn_s_memrealtime();
        if (!fuse && ev == 0) pidx_apply(a.nbr, a.tailinc, a.cnt[C_NPAIR], qi, a.map, a.pbkt, a.map_cap);
        // wait until no partial of this evaluation is the sentinel any more (threads t < 30 poll
        // their product over the 32 chunks); after kLmStealPolls rounds, claim and reduce chunks
        // nobody has claimed (their home workgroups have not started)
        const double* P = a.part + (size_t)ev * kLmBlocks * 32;
        const unsigned long long t0 = rt_now();
        double pv[kLmBlocks];
        for (unsigned polls = 0;; ++polls) {
            bool ok = true;
            if (t < kLmParts) {
#pragma unroll
                for (int b = 0; b < kLmBlocks; ++b)
                    pv[b] = __hip_atomic_load(P + 32 * b + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int b = 0; b < kLmBlocks; ++b) ok = ok && __double_as_longlong(pv[b]) != (long long)kPartSentinel;
            }
            if (__syncthreads_and(ok)) break;
            if (t == 0) {
                s_state = 0;
                if (polls >= kLmStealPolls) {
                    const u32 m = __hip_atomic_load(&claim[ev], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (m != kFull) {
                        const int c = __ffs(~m & kFull) - 1;
                        const u32 o2 = __hip_atomic_fetch_or(&claim[ev], 1u << c, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
                        if (!((o2 >> c) & 1u)) {
                            s_steal = c;
                            s_state = 2;
                        }
                    }
                }
                if (s_state == 0 && rt_now() - t0 > kWaitTicks) {
                    aborted = 1;
                    a.cnt[C_ERR] = 1;
                    atomicOr(a.err, 1);
                }
            }
            __syncthreads();
            if (aborted) break;
            if (s_state == 2) {
                if (fuse && ev == 0) observe_chunk(s_steal, false);   // the chunk's observe pass is ours
                reduce_chunk(s_steal, ev, 0u, false);
            } else {
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (aborted) break;
        if (rec) dbg[3 + 4 * ev] = __builtin_amdgcn_s_memrealtime();
        if (recb) recb[2 * (ev * kLmBlocks + blockIdx.x) + 1] = __builtin_amdgcn_s_memrealtime();
        if (t < kLmParts) {
            double v = 0.0;
#pragma unroll
            for (int b = 0; b < kLmBlocks; ++b) v += pv[b];
            tot[t] = v;
        }
        __syncthreads();
        if (fuse && ev == 0) {                                   // the residual count (kept rows)
            const int nr = (int)tot[kLmParts - 1];
            if (nr == 0) {                                       // no residual blocks: untouched
                apply_commits(t, 256);
                if (a.prep.on) rgm_prep_apps<NC>(a.prep, a.cnt, a.st->params);
                return;
            }
            if (t == 0) lm.n_res = nr;
            // a home chunk another workgroup claimed first (this one started late): its observe pass
            // here may have read g bytes that were already incremented, so the kept bits are re-read
            // from the claimant's commits, complete since its partials arrived
            if ((old0 >> blockIdx.x) & 1u) s_mine[t] = load_res((int)blockIdx.x * 256 + t);
        }
        if (rec) dbg[40 + ev] = __builtin_amdgcn_s_memrealtime();
        if (t < 2) {                                             // lanes 0 and 1, identical state
            LmCore c;
            unsigned long long* pr = (rec && ev == 1) ? dbg + 21 : nullptr;
            core_load(c, lm);
            if (pr) pr[4] = __builtin_amdgcn_s_memrealtime();
            lm_accept(c, tot, lm.best, pr);
            if (pr) pr[3] = __builtin_amdgcn_s_memrealtime();
            if (ev == kLmEvals - 1) c.done = 1;
            if (t == 0) core_store(c, lm);
        } else if (fuse && ev == 0 && t >= 64) {
            apply_commits(t - 64, 192);                          // waves 1-3, beside the serial step
        }
        if (fuse && ev == 0) applied = true;
        __syncthreads();
        if (rec) dbg[4 + 4 * ev] = __builtin_amdgcn_s_memrealtime();
    }
    if (!applied) apply_commits(t, 256);
    if (blockIdx.x == 0 && t == 0) {
        for (int k = 0; k < 7; ++k) a.st->params[k] = lm.best[k];
        atomicAdd(&a.cnt[C_LM_ITERS], lm.iteration);
        *a.lm_out = lm;
    }
    if (a.prep.on) rgm_prep_apps<NC>(a.prep, a.cnt, lm.best);   // every workgroup holds the solution
}

// ---------------------------------- pose / map update ---------------------------------------
// mode 1: odom = (q2m(q), t) from the solved pose (:278-280); mode 0: keep odom. Writes the pose
// {m2q(odom.rotation()), odom.translation()} of the node (copy.cpp:105-107).
__device__ __forceinline__ void finalize_pose(DevState* st, double* poses, int pose_cap, int mode, u32* acc,
                                              const double* prm) {
    const int t = threadIdx.x;
    if (t != 0) return;
    if (mode == 1) {
        const qd q{prm[0], prm[1], prm[2], prm[3]};
        iso o;
        o.R = q2m(q);
        o.t = d3{prm[4], prm[5], prm[6]};
        store_iso(o, st->odomR, st->odomt);
    }
    const iso o = load_iso(st->odomR, st->odomt);
    const qd q = m2q(polar_rotation(o.R));
    double* P = poses + 7 * (size_t)(st->frame % pose_cap);
    P[0] = q.x; P[1] = q.y; P[2] = q.z; P[3] = q.w;
    P[4] = o.t.x; P[5] = o.t.y; P[6] = o.t.z;
    st->frame++;
}

__global__ void k_finalize(DevState* __restrict__ st, double* __restrict__ poses, int pose_cap, int mode,
                           u32* __restrict__ acc) {
    double prm[7];
    for (int k = 0; k < 7; ++k) prm[k] = st->params[k];
    finalize_pose(st, poses, pose_cap, mode, acc, prm);
}


// CropBox bounds t +- 100 as float, inclusive (:606-615, B.2)
__device__ __forceinline__ bool in_crop(const DevState* st, float4 p) {
    const float lox = (float)(st->odomt[0] - 100), loy = (float)(st->odomt[1] - 100), loz = (float)(st->odomt[2] - 100);
    const float hix = (float)(st->odomt[0] + 100), hiy = (float)(st->odomt[1] + 100), hiz = (float)(st->odomt[2] + 100);
    return !((p.x < lox || p.y < loy || p.z < loz) || (p.x > hix || p.y > hiy || p.z > hiz));
}

// addPointsToMap, first pass: the pose (:278-280, k_finalize mode 1, by thread 0 of block 0), the
// transform / append of the down-sampled clouds (:592-604, r and g carried) and the CropBox-kept
// min / max of every class for the rgbds grids (:606-615, :40-51). The crop box is odom.t +- 100,
// and odom.t is the solved translation params[4..6] that the pose step stores. The pose step (a
// single-thread SVD polar factor, finalize_pose) runs on the grid's last workgroup, which takes no
// part in the points, so it overlaps them instead of delaying block 0's share.
template <int NC>
__global__ void __launch_bounds__(256) k_rg_append_minmax(DevState* __restrict__ st, int* __restrict__ cnt,
                                                           u32* __restrict__ acc, Clouds map, Clouds ds,
                                                           CloudsW app, double* __restrict__ poses, int pose_cap) {
    double prm[7];
    for (int k = 0; k < 7; ++k) prm[k] = st->params[k];
    if (blockIdx.x == gridDim.x - 1) {
        finalize_pose(st, poses, pose_cap, 1, acc, prm);
        return;
    }
    const int nblk = (int)gridDim.x - 1;
    const float lox = (float)(prm[4] - 100), loy = (float)(prm[5] - 100), loz = (float)(prm[6] - 100);   // in_crop
    const float hix = (float)(prm[4] + 100), hiy = (float)(prm[5] + 100), hiz = (float)(prm[6] + 100);
    constexpr int nc = NC;
    const RgView<NC> V = rg_view<NC>(cnt, map, Clouds{{app.p[0], app.p[1], app.p[2]}});
    const int n = V.total();
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[C_NRG] = n;
    float v[6 * kMaxC];
    minmax_init(v);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nblk * blockDim.x) {
        int c, li;
        bool ap;
        V.locate(i, c, li, ap);
        float4 p;
        if (ap) {                                      // appended: pointAssociateToMap of the ds point
            p = associate(prm, ds.at(c)[li]);
            app.at(c)[li] = p;
        } else {
            p = map.at(c)[li];
        }
        if ((p.x < lox || p.y < loy || p.z < loz) || (p.x > hix || p.y > hiy || p.z > hiz)) continue;
        minmax_add(v, c, p);
    }
    minmax_commit(v, acc + A_RG, nc);
}

// ---- order-free voxel groups of the tie-order rgbds (the heap tier's dependence flags, pf_tie.h) ----
// The reference sums a voxel's points in the order std::sort leaves them (:108-125), so the tie order is
// observable only through groups whose f32 sum depends on that order: a group of one or two points is
// order-free (0 + a is exact and + commutes), a group of three is order-free when its three left folds
// ((0 + a) + b) + c, ((0 + a) + c) + b and ((0 + b) + c) + a agree bit for bit in x, y and z (the first two
// terms commute), and a larger group counts as order-dependent. The key kernels insert elements into an
// open-addressing table (key -> count and the first three elements), k_rg_dep decides every group from
// its slot, marks its members and empties the slot for the next update.
// The map an rgbds writes holds one centroid per voxel, so two map points share a voxel only when a
// centroid rounds across a voxel face (k_rg_tail checks every kept centroid against its voxel) or the
// host wrote the map (initMapWithPoints, set_map, restore, the switch into this order). While neither
// happened (dirty[0] == 0, k_rg_write moves k_rg_tail's verdict there) a group of three or more holds at
// least two appended points, so only the appended points (a few thousand) go into a small table (the
// first 2^kDepSmallBits slots) and the map points only probe it (k_rg_dep_probe, read-only unless their
// voxel is there): configs[4]'s 2M-point map no longer inserts two million elements per frame.
struct DepTab {
    u32* key;
    u32* cnt;
    u32* mem;
    u32* slot;
    u8* freef;
    u32 hbits;
    u32* dirty;          // [0]: the map may hold two points of one voxel; [1]: k_rg_tail's verdict
};
constexpr u32 kDepEmpty = 0xFFFFFFFFu;
constexpr u32 kDepSmallBits = 16;
constexpr int kDepSmallApp = 1 << (kDepSmallBits - 2);   // appended points the small table takes

// this update's table: the small one (clean map, few appended points) or the full one
template <int NC>
__device__ __forceinline__ bool dep_small(const DepTab& T, const int* cnt) {
    if (!T.key || !T.dirty || T.dirty[0] != 0u || T.hbits < kDepSmallBits) return false;
    int na = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) na += cnt[C_DS + c];
    return na <= kDepSmallApp;
}

__device__ __forceinline__ u32 dep_hash(u32 key, u32 bits) { return (key * 0x9E3779B1u) >> (32u - bits); }

__device__ __forceinline__ void dep_insert(const DepTab& T, u32 key, u32 e, bool small = false) {
    if (!T.key) return;
    if (key == kSentinel) {                        // cropped: in no voxel
        T.slot[e] = kDepEmpty;
        T.freef[e] = 1;
        return;
    }
    const u32 bits = small ? kDepSmallBits : T.hbits;
    const u32 mask = (1u << bits) - 1u;
    u32 sl = dep_hash(key, bits);
    for (;;) {
        const u32 old = atomicCAS(&T.key[sl], kDepEmpty, key);
        if (old == kDepEmpty || old == key) break;
        sl = (sl + 1u) & mask;
    }
    const u32 c = atomicAdd(&T.cnt[sl], 1u);
    if (c < 3u) T.mem[3u * sl + c] = e;
    T.slot[e] = sl;
    T.freef[e] = 0;
}

// an element of the key kernels: appended points always go into the table, map points only when the
// map may hold two points of a voxel (otherwise k_rg_dep_probe looks them up)
__device__ __forceinline__ void dep_element(const DepTab& T, u32 key, u32 e, bool appended, bool small) {
    if (!T.key) return;
    if (small && !appended) {
        T.slot[e] = kDepEmpty;
        T.freef[e] = 1;
        return;
    }
    dep_insert(T, key, e, small);
}

__device__ __forceinline__ bool folds_agree(float4 a, float4 b, float4 c) {
    const float A[3] = {a.x, a.y, a.z}, B[3] = {b.x, b.y, b.z}, C[3] = {c.x, c.y, c.z};
    bool same = true;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float f1 = ((0.f + A[d]) + B[d]) + C[d];
        const float f2 = ((0.f + A[d]) + C[d]) + B[d];
        const float f3 = ((0.f + B[d]) + C[d]) + A[d];
        same = same && __float_as_uint(f1) == __float_as_uint(f2) && __float_as_uint(f1) == __float_as_uint(f3);
    }
    return same;
}

// the small table's map members: a map point joins the group of its voxel when appended points are there
template <int NC>
__global__ void __launch_bounds__(256) k_rg_dep_probe(const int* __restrict__ cnt, const u32* __restrict__ keys,
                                                      DepTab T) {
    if (!dep_small<NC>(T, cnt)) return;
    const RgView<NC> V = rg_view<NC>(cnt, Clouds{}, Clouds{});
    const int n = V.total();
    const u32 mask = (1u << kDepSmallBits) - 1u;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        int c, li;
        bool ap;
        V.locate(e, c, li, ap);
        const u32 key = keys[e];
        if (ap || key == kSentinel) continue;
        u32 sl = dep_hash(key, kDepSmallBits);
        for (;;) {
            const u32 k = T.key[sl];
            if (k == kDepEmpty) break;
            if (k == key) {
                const u32 m = atomicAdd(&T.cnt[sl], 1u);
                if (m < 3u) T.mem[3u * sl + m] = (u32)e;
                T.slot[e] = sl;
                T.freef[e] = 0;
                break;
            }
            sl = (sl + 1u) & mask;
        }
    }
}

// decides every group of the table: one thread per group
template <int NC>
__device__ __forceinline__ void dep_decide(const DepTab& T, const RgView<NC>& V, u32 sl) {
    const u32 c = T.cnt[sl];
    bool fre = c <= 2u;
    if (c == 3u) {
        int cc;
        const float4 a = V.at((int)T.mem[3u * sl], cc), b = V.at((int)T.mem[3u * sl + 1u], cc),
                     d = V.at((int)T.mem[3u * sl + 2u], cc);
        fre = folds_agree(a, b, d);
    }
    if (fre)
        for (u32 j = 0; j < c; ++j) T.freef[T.mem[3u * sl + j]] = 1;
    T.key[sl] = kDepEmpty;
    T.cnt[sl] = 0u;
}

template <int NC>
__global__ void __launch_bounds__(256) k_rg_dep(const int* __restrict__ cnt, Clouds map, Clouds app, DepTab T) {
    const RgView<NC> V = rg_view<NC>(cnt, map, app);
    if (dep_small<NC>(T, cnt)) {                   // the small table's slots
        for (u32 sl = blockIdx.x * blockDim.x + threadIdx.x; sl < (1u << kDepSmallBits); sl += gridDim.x * blockDim.x)
            if (T.key[sl] != kDepEmpty) dep_decide(T, V, sl);
        return;
    }
    const int n = V.total();
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        const u32 sl = T.slot[e];
        if (sl == kDepEmpty || T.mem[3u * sl] != (u32)e) continue;   // only the group's first element
        dep_decide(T, V, sl);
    }
}

template <int NC>
__global__ void __launch_bounds__(256) k_rg_keys(const DevState* __restrict__ st, const int* __restrict__ cnt,
                                                  const u32* __restrict__ acc, Clouds map, Clouds app,
                                                  VgLeaf leaf, u32* __restrict__ keys, u32* __restrict__ vals,
                                                  SortHist sh, DepTab dt) {
    __shared__ u32 lh[4][256];
    sort_hist_begin(lh);
    const RgView<NC> V = rg_view<NC>(cnt, map, app);
    const int n = V.total();
    const bool small = dep_small<NC>(dt, cnt);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        int c;
        const float4 p = V.at(i, c);
        vals[i] = (u32)i;
        if (!in_crop(st, p)) {
            keys[i] = kSentinel;
            sort_hist_add(lh, kSentinel, sh.passes);
            dep_element(dt, kSentinel, (u32)i, false, false);
            continue;
        }
        const float lf = leaf.at(c);
        const u32* a = acc + A_RG + 6 * c;
        int minb[3], div[3];
        for (int k = 0; k < 3; ++k) {                                // :46-56 (f32 division)
            minb[k] = (int)floorf(ord2f(a[k]) / lf);
            div[k] = (int)floorf(ord2f(a[3 + k]) / lf) - minb[k] + 1;
        }
        const int i0 = (int)(floorf(p.x / lf) - (float)minb[0]);  // :63-65
        const int i1 = (int)(floorf(p.y / lf) - (float)minb[1]);
        const int i2 = (int)(floorf(p.z / lf) - (float)minb[2]);
        const int idx = i0 * 1 + i1 * div[0] + i2 * (div[0] * div[1]);
        keys[i] = ((u32)idx & 0x3fffffffu) | ((u32)c << 30);
        sort_hist_add(lh, keys[i], sh.passes);
        int cc, li;
        bool ap;
        V.locate(i, cc, li, ap);
        dep_element(dt, keys[i], (u32)i, ap, small);
    }
    sort_hist_end(lh, sh, n, n);
}

// addPointsToMap's first pass and the rgbds keys in one launch, when the crop box bounds the key
// grid (rg_fused_keys): the rgbds grid of the reference starts at the voxel of the kept points'
// minimum (:40-56), but the sort only needs the keys' order, and idx = i0 + div0 (i1 + div1 i2) with
// 0 <= i < div orders voxels lexicographically by (i2, i1, i0) for any origin at or below the minimum
// and any extent covering the maximum. The crop box t +- 100 is such a box (kept points satisfy
// lo <= p <= hi, and fl(p / leaf) and floor are monotone), so keys taken on its voxel grid sort the
// points exactly as the reference's do, equal keys being the same voxels: no min / max pass, no
// second launch. Pose step on the last workgroup as in k_rg_append_minmax.
template <int NC>
__global__ void __launch_bounds__(256) k_rg_append_keys(DevState* __restrict__ st, int* __restrict__ cnt,
                                                         u32* __restrict__ acc, Clouds map, Clouds ds, CloudsW app,
                                                         double* __restrict__ poses, int pose_cap, VgLeaf leaf,
                                                         u32* __restrict__ keys, u32* __restrict__ vals,
                                                         SortHist sh, DepTab dt) {
    double prm[7];
    for (int k = 0; k < 7; ++k) prm[k] = st->params[k];
    if (blockIdx.x == gridDim.x - 1) {
        finalize_pose(st, poses, pose_cap, 1, acc, prm);
        return;                                    // holds no keys: not counted by sort_hist_end
    }
    __shared__ u32 lh[4][256];
    sort_hist_begin(lh);
    const int nblk = (int)gridDim.x - 1;
    const float lo[3] = {(float)(prm[4] - 100), (float)(prm[5] - 100), (float)(prm[6] - 100)};   // in_crop
    const float hi[3] = {(float)(prm[4] + 100), (float)(prm[5] + 100), (float)(prm[6] + 100)};
    const RgView<NC> V = rg_view<NC>(cnt, map, Clouds{{app.p[0], app.p[1], app.p[2]}});
    const int n = V.total();
    const bool small = dep_small<NC>(dt, cnt);
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[C_NRG] = n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nblk * blockDim.x) {
        int c, li;
        bool ap;
        V.locate(i, c, li, ap);
        float4 p;
        if (ap) {                                      // appended: pointAssociateToMap of the ds point
            p = associate(prm, ds.at(c)[li]);
            app.at(c)[li] = p;
        } else {
            p = map.at(c)[li];
        }
        vals[i] = (u32)i;
        u32 key = kSentinel;
        if (!((p.x < lo[0] || p.y < lo[1] || p.z < lo[2]) || (p.x > hi[0] || p.y > hi[1] || p.z > hi[2]))) {
            const float lf = leaf.at(c);
            int minb[3], div[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                minb[k] = (int)floorf(lo[k] / lf);
                div[k] = (int)floorf(hi[k] / lf) - minb[k] + 1;
            }
            const int i0 = (int)(floorf(p.x / lf) - (float)minb[0]);
            const int i1 = (int)(floorf(p.y / lf) - (float)minb[1]);
            const int i2 = (int)(floorf(p.z / lf) - (float)minb[2]);
            const int idx = i0 * 1 + i1 * div[0] + i2 * (div[0] * div[1]);
            key = ((u32)idx & 0x3fffffffu) | ((u32)c << 30);
        }
        keys[i] = key;
        sort_hist_add(lh, key, sh.passes);
        dep_element(dt, key, (u32)i, ap, small);
    }
    const int items = n < nblk * 256 ? n : nblk * 256;  // blocks holding keys: the first ceil(items / 256)
    sort_hist_end(lh, sh, n, items);
}

// whether the crop box's voxel grid of every class fits the 30 key bits (k_rg_append_keys); the
// extent is at most floor(200 / leaf) + 2 voxels per axis
inline bool rg_fused_keys(const float* leaf, int nc) {
    for (int c = 0; c < nc; ++c) {
        const double d = std::floor(200.0 / (double)leaf[c]) + 3.0;
        if (!(d * d * d < (double)(1u << 30))) return false;
    }
    return true;
}

struct RgTailArgs {
    int* cnt;
    Clouds map, app;
    const u32* keys;       // sorted (bits 30-31 class, 0xFFFFFFFF cropped), cnt[C_NRG] of them
    const u32* vals;
    float4* seg_out;       // the kept voxels, compacted in key order
    int k_new;
    float theta_p;
    int theta_max;
    u64* status;           // look-back words (zero between calls)
    u32* arrive;
    int* err;
    VgLeaf leaf;           // the classes' voxel sizes (the centroid check)
    u32* dirty;            // DepTab::dirty (tie order) or null: [1] |= a kept centroid left its voxel
};

// The rest of addPointsToMap in one pass over the sorted keys (one tile of 256 x kTailPer keys per
// workgroup turn, kTailPer consecutive keys per thread, their points loaded at once): every voxel (segment of equal keys) is reduced by the thread holding
// its first key, walking its points in key order (the Vector4f centroid and r / g maxima of :108-125,
// extractstablepoint :12-14, the ageing :634-646); the kept voxels are counted per tile and a
// decoupled look-back over the tile counts gives each kept voxel its place in seg_out, so segment
// starts, their reduction, the keep-flag scan and the compaction need no separate launches.
// cnt[C_NLT + b - 1] = kept voxels of classes < b, cnt[C_KEEP_TOTAL] = all kept voxels.
#ifndef PF_RG_TAIL_PER
#define PF_RG_TAIL_PER 2
#endif
constexpr int kTailPer = PF_RG_TAIL_PER;                        // keys per thread
constexpr int kTailTile = 256 * kTailPer;
template <int NC>
__global__ void __launch_bounds__(256) k_rg_tail(RgTailArgs a) {
    constexpr u32 kSent = 0xFFFFFFFFu;
    constexpr int kPer = kTailPer;
    __shared__ u32 lw[4];
    __shared__ u32 s_excl;
    const RgView<NC> V = rg_view<NC>(a.cnt, a.map, a.app);
    int* kb = a.cnt + C_NLT;
    const int n = a.cnt[C_NRG];
    const int ntiles = (n + kTailTile - 1) / kTailTile;
    const int t = threadIdx.x;
    const int G = ntiles < (int)gridDim.x ? ntiles : (int)gridDim.x;
    if (n == 0) {
        if (blockIdx.x == 0 && t == 0) {
            a.cnt[C_KEEP_TOTAL] = 0;
            kb[0] = kb[1] = kb[2] = 0;
        }
        return;
    }
    if ((int)blockIdx.x >= G) return;
    if (blockIdx.x == 0 && t == 0) {                            // classes below the first key's: none
        const u32 k0 = a.keys[0];
        for (u32 b = 1; b <= 3; ++b)
            if ((k0 >> 30) >= b) kb[b - 1] = 0;
    }
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int base = tile * kTailTile + t * kPer;
        u32 k[kPer + 1];                                        // k[0] = predecessor of the first
        k[0] = base > 0 && base - 1 < n ? a.keys[base - 1] : kSent;
#pragma unroll
        for (int j = 0; j < kPer; ++j) k[j + 1] = base + j < n ? a.keys[base + j] : kSent;
        float4 pt[kPer];                                        // this thread's points, loaded at once
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            int c;
            pt[j] = base + j < n && k[j + 1] != kSent ? V.at((int)a.vals[base + j], c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float4 out[kPer];
        u32 keepm = 0u;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = base + j;
            out[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!(i < n && k[j + 1] != kSent && (i == 0 || k[j] != k[j + 1]))) continue;   // not a voxel's first key
            float cx = 0.f, cy = 0.f, cz = 0.f;                 // Vector4f centroid (:108-125)
            int r_max = -1;
            float g_max = -1;
            int e = i;
            float4 p0 = make_float4(0.f, 0.f, 0.f, 0.f);        // the voxel's first point
            for (;;) {
                float4 p;
                if (e - base < kPer) {
#pragma unroll
                    for (int jj = 0; jj < kPer; ++jj)           // static register index
                        if (jj == e - base) p = pt[jj];
                } else {                                        // the voxel runs past this thread's keys
                    int c;
                    p = V.at((int)a.vals[e], c);
                }
                if (e == i) p0 = p;
                cx += p.x; cy += p.y; cz += p.z;
                const int r = (int)w_r(p);
                const float g = (float)w_g(p);
                if (r > r_max) r_max = r;
                if (g > g_max) g_max = g;
                if (++e >= n) break;
                const u32 ke = e - base < kPer ? k[e - base + 1] : a.keys[e];
                if (ke != k[j + 1]) break;
            }
            const float nn = (float)(e - i);
            const u32 r = (u32)r_max & 255u, g = (u32)g_max & 255u;     // stored into uint8 r, g
            // extractstablepoint (:12-14) on the voxel's uint8 r, g
            const bool drop = ((float)g < (float)r * a.theta_p) && ((int)r > a.k_new) && ((int)g < a.theta_max + 1);
            const u32 aged = r > 250 ? 255u : r + 2u;                   // :634-646
            out[j] = make_float4(cx / nn, cy / nn, cz / nn, __uint_as_float(pack_rg(aged, g)));
            if (!drop) keepm |= 1u << j;
            if (!drop && a.dirty) {                             // the centroid's voxel, keyed as the next update will
                const float lf = a.leaf.at((int)(k[j + 1] >> 30));
                if (floorf(out[j].x / lf) != floorf(p0.x / lf) || floorf(out[j].y / lf) != floorf(p0.y / lf) ||
                    floorf(out[j].z / lf) != floorf(p0.z / lf))
                    atomicOr(a.dirty + 1, 1u);
            }
        }
        u32 agg;
        const u32 tex = block_excl_scan256((u32)__popc(keepm), lw, agg);
        if (t < 64) {
            const u32 excl = tile_lookback(a.status, tile, agg, a.err);
            if (t == 0) {
                s_excl = excl;
                if (tile == ntiles - 1) {
                    a.cnt[C_KEEP_TOTAL] = (int)(excl + agg);
                    for (u32 b = 1; b <= 3; ++b)                // classes above the last key's: all
                        if ((a.keys[n - 1] >> 30) < b) kb[b - 1] = (int)(excl + agg);
                }
            }
        }
        __syncthreads();
        u32 pos = s_excl + tex;                                 // kept voxels before key base + j
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = base + j;
            if (i >= n) break;
            const u32 kp = k[j], kc = k[j + 1];
            if (i > 0 && (kp >> 30) < (kc >> 30))              // class boundary: kept voxels before it
                for (u32 b = (kp >> 30) + 1; b <= (kc >> 30); ++b) kb[b - 1] = (int)pos;
            if ((keepm >> j) & 1u) a.seg_out[pos++] = out[j];
        }
        __syncthreads();
    }
    lookback_finish(a.status, ntiles, a.arrive, G);
}

// the kept voxels into the class maps (class c's are seg_out[kb(c) .. kb(c + 1)), in order)
template <int NC>
__global__ void __launch_bounds__(256) k_rg_write(int* __restrict__ cnt, const float4* __restrict__ seg_out,
                                                   CloudsW map, u32* __restrict__ dirty) {
    constexpr int nc = NC;
    const int total = cnt[C_KEEP_TOTAL];
    if (dirty && blockIdx.x == 0 && threadIdx.x == 0) {   // k_rg_tail's verdict on the map written here
        dirty[0] = dirty[1];
        dirty[1] = 0u;
    }
    int kb[kMaxC + 1];                             // kept-voxel start of every class
    kb[0] = 0;
#pragma unroll
    for (int c = 1; c <= kMaxC; ++c) kb[c] = c < nc ? cnt[C_NLT + c - 1] : total;
    if (blockIdx.x == 0 && threadIdx.x == 0)      // no block of this kernel reads them
        for (int c = 0; c < nc; ++c) cnt[C_M + c] = kb[c + 1] - kb[c];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int c = NC == 2 ? (i < kb[1] ? 0 : 1) : (i < kb[1] ? 0 : (i < kb[2] ? 1 : 2));
        map.at(c)[i - sel3(c, kb[0], kb[1], kb[2])] = seg_out[i];
    }
}

// ---------------------------- rgbds by merge (the default order) ----------------------------
// addPointsToMap's rgbds (:606-626, :34-134) orders the elements (map points, then this frame's
// appended points, per class) by voxel index and, within a voxel, by element index (the stable order;
// the reference-tie-order mode keeps the radix path above), then reduces every voxel. The voxel index
// orders voxels lexicographically by (z, y, x) on any grid covering the points (k_rg_append_keys), so
// the 64-bit key class << 62 | z << 40 | y << 20 | x of the voxel coordinates (20 bits each, biased)
// orders them the same way on every frame. The map the previous rgbds wrote is already in that order
// (its points are voxel centroids written in key order), so the map's own keys split the key range into
// kRgmBuckets buckets of equal map-point counts, and one workgroup per bucket does all of its work:
// it keys its map points and checks their order; scans every appended point (pointAssociateToMap
// :592-604), keeping those of its bucket and counting those below it; sorts its appended points by
// (key, element) in registers and LDS (a bitonic network, shuffles within a wave); reduces the voxels
// of its bucket (the Vector4f centroid and r / g maxima of :108-125, extractstablepoint :12-14, the
// ageing :634-646, cropped elements skipped); ranks the kept voxels in merged order and writes them
// and publishes its length and kept voxels per class. k_rgm_finish (a second launch, one workgroup per
// bucket) then writes each bucket's kept voxels into the other map set (mapset[mpar ^ 1]) at their
// class-map index and the map sizes. No workgroup of a launch waits on another (a look-back across
// buckets deadlocked when many handles' launches shared the CUs: nothing guarantees that the bucket a
// workgroup waits on is resident). When the map is not in key order (the first update after
// initMapWithPoints or pf_odom_set_map, or a centroid that rounded into a neighbouring voxel) or a
// bucket holds more than kRgmBucketCap appended points, the buckets' output is void and k_rgm_finish's
// workgroup 0 sorts every element (a stable LSD radix sort over the 64-bit keys) and reduces the voxels
// itself.

struct RgmArgs {
    DevState* st;
    int* cnt;
    u32* acc;
    Clouds map, ds;
    CloudsW app;
    double* poses;
    int pose_cap;
    VgLeaf leaf;
    int k_new;
    float theta_p;
    int theta_max;
    u64* okey;             // [map points] keys, map order
    u64* key64;            // [elements] keys, element order (for the fallback)
    u32* vtag;             // [elements] element | cropped << 31
    float4* vox;           // [elements] a voxel's output at its merged position
    u32* kflag;            // [elements] class << 30 | kept flag, then class << 30 | rank + 1, at merged positions
    CloudsW mapw;          // the new class maps (the other map set)
    u32 map_cap;
    int* err_map;          // sticky error word E_MAP
    u64* kout;             // fallback: sorted keys / tags and scratch
    u32* vout;
    u64* ktmp;
    u32* vtmp;
    int* stat;             // [8] (OdomGPU::rgm_stat)
    int* bmeta;            // [kRgmBuckets][kRgmMeta]: merged base, length, kept voxels per class, and the
                           // cell bounds of its kept voxels per class (min x y z, max x y z) (-> k_rgm_finish)
    int* gdims;            // the next update's map grid: dims, scan length, error word (grid_dims)
    int* gncells;
    long long gcell_cap;
    int* gerr;
    u32* bcount;           // the appended points' bucket lists (RgmPrep)
    const u64* bkey;
    const u32* btag;
    unsigned long long* dbg;   // development probe (PF_PROBE): [64 + 10 b + i] phase timestamps of bucket b
};
static_assert(64 + 10 * (kRgmBuckets + 1) <= kLmBlkProbe, "probe words");
constexpr int kRgmMeta = 32;                           // ints per bucket in bmeta
constexpr int kRgmBnd = 8;                             // bmeta offset of the bounds

// per-class cell bounds (the grid's 1 m cells, as k_grid_bounds computes them) in LDS
__device__ __forceinline__ void rgm_bound_init(int (*bnd)[6], int t) {
    if (t < 6 * kMaxC) bnd[t / 6][t % 6] = (t % 6) < 3 ? INT_MAX : INT_MIN;
}
__device__ __forceinline__ void rgm_bound_add(int (*bnd)[6], int c, float4 p) {
    const int x = (int)floorf(p.x), y = (int)floorf(p.y), z = (int)floorf(p.z);
    atomicMin(&bnd[c][0], x); atomicMin(&bnd[c][1], y); atomicMin(&bnd[c][2], z);
    atomicMax(&bnd[c][3], x); atomicMax(&bnd[c][4], y); atomicMax(&bnd[c][5], z);
}

// one voxel of rgbds: the f32 centroid of its points in order and the maxima of r and g (:108-125),
// then extractstablepoint (:12-14) and the ageing (:634-646)
struct RgmVox {
    float cx = 0.f, cy = 0.f, cz = 0.f;
    int r_max = -1;
    float g_max = -1;
    int n = 0;
    __device__ __forceinline__ void add(float4 p) {
        cx += p.x; cy += p.y; cz += p.z;
        const int r = (int)w_r(p);
        const float g = (float)w_g(p);
        if (r > r_max) r_max = r;
        if (g > g_max) g_max = g;
        ++n;
    }
    // the output point; returns whether the voxel is kept
    __device__ __forceinline__ bool finish(int k_new, float theta_p, int theta_max, float4& out) const {
        const float nn = (float)n;
        const u32 r = (u32)r_max & 255u, g = (u32)g_max & 255u;     // stored into uint8 r, g
        const bool drop = ((float)g < (float)r * theta_p) && ((int)r > k_new) && ((int)g < theta_max + 1);
        const u32 aged = r > 250 ? 255u : r + 2u;
        out = make_float4(cx / nn, cy / nn, cz / nn, __uint_as_float(pack_rg(aged, g)));
        return !drop;
    }
};

// exclusive scan across a 1024-thread block (lds: 16 words)
__device__ __forceinline__ u32 block_excl_scan1024(u32 v, u32* lds, u32& total) {
    const int w = threadIdx.x >> 6, l = lane_id();
    const u32 inc = wave_incl_scan_u32(v);
    if (l == 63) lds[w] = inc;
    __syncthreads();
    u32 off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kRgmThreads / 64; ++i) {
        const u32 x = lds[i];
        if (i < w) off += x;
        tot += x;
    }
    __syncthreads();
    total = tot;
    return off + inc - v;
}

// block b < kRgmBuckets: bucket b (map points [lo, hi) = [b M / R, (b + 1) M / R), appended points
// whose key lies in [key(lo), key(hi))); block kRgmBuckets: the pose step (as in k_rg_append_keys)
// Bitonic sort of bk / bt[0 .. cb) (cb <= E * 1024) by (key, element), E elements per thread in
// registers: element e of thread t is index e * 1024 + t, so partners at distance >= 1024 are in the
// same thread (register compare), at 64 .. 512 in another wave (through LDS, two barriers), below 64 in
// the same wave (shuffles)
template <int E>
__device__ __forceinline__ void rgm_sort_regs(u64* bk, u32* bt, int cb) {
    const int t = threadIdx.x;
    // one element per thread: the network of the next power of two >= cb (at least a wave); threads
    // past it hold padding and only meet padding
    int S = E * kRgmThreads;
    if (E == 1) {
        S = 64;
        while (S < cb) S <<= 1;
    }
    u64 k[E];
    u32 g[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = e * kRgmThreads + t;
        k[e] = i < cb ? bk[i] : ~0ull;
        g[e] = i < cb ? bt[i] : ~0u;
    }
    __syncthreads();
    for (int kk = 2; kk <= S; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j >= kRgmThreads) {
                const int je = j / kRgmThreads;
#pragma unroll
                for (int e = 0; e < E; ++e)
#pragma unroll
                    for (int e2 = e + 1; e2 < E; ++e2) {           // static register indices
                        if ((e & je) || e2 != (e | je)) continue;
                        const bool up = ((e * kRgmThreads + t) & kk) == 0;
                        const bool sw = up ? rgm_less(k[e2], g[e2], k[e], g[e]) : rgm_less(k[e], g[e], k[e2], g[e2]);
                        if (sw) {
                            const u64 tk = k[e]; k[e] = k[e2]; k[e2] = tk;
                            const u32 tg = g[e]; g[e] = g[e2]; g[e2] = tg;
                        }
                    }
                continue;
            }
            u64 pk[E];
            u32 pg[E];
            if (j < 64) {
                if (E == 1 && t >= S) continue;             // padding waves (wave-uniform: S >= 64)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const u32 lo32 = (u32)__shfl_xor((int)(u32)k[e], j, 64);
                    const u32 hi32 = (u32)__shfl_xor((int)(u32)(k[e] >> 32), j, 64);
                    pk[e] = ((u64)hi32 << 32) | lo32;
                    pg[e] = (u32)__shfl_xor((int)g[e], j, 64);
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    bk[e * kRgmThreads + t] = k[e];
                    bt[e * kRgmThreads + t] = g[e];
                }
                __syncthreads();
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    pk[e] = bk[e * kRgmThreads + (t ^ j)];
                    pg[e] = bt[e * kRgmThreads + (t ^ j)];
                }
                __syncthreads();
            }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int i = e * kRgmThreads + t;
                const bool up = (i & kk) == 0, lower = (t & j) == 0;
                const bool pless = rgm_less(pk[e], pg[e], k[e], g[e]);
                // the lower index of an ascending pair keeps the smaller element
                if ((lower == up) ? pless : !pless && !(pk[e] == k[e] && pg[e] == g[e])) {
                    k[e] = pk[e];
                    g[e] = pg[e];
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        bk[e * kRgmThreads + t] = k[e];
        bt[e * kRgmThreads + t] = g[e];
    }
}

#define RGM_MARK(i)                                                                              \
    do {                                                                                         \
        if (a.dbg && t == 0) a.dbg[64 + 10 * b + (i)] = __builtin_amdgcn_s_memrealtime();        \
    } while (0)
template <int NC>
__global__ void __launch_bounds__(kRgmThreads) k_rgm_bucket(RgmArgs a) {
    __shared__ u64 bk[kRgmBucketCap];
    __shared__ u32 bt[kRgmBucketCap];
    __shared__ u64 ok[kRgmOldLds];
    __shared__ float4 opt[kRgmOldLds];                 // the bucket's map points (when cached)
    __shared__ float4 apt[kRgmAppLds];                 // its appended points in sorted order (when cached)
    __shared__ u64 s_nextk;
    __shared__ int s_cnt, s_before[kRgmThreads / 64], s_cls[kMaxC];
    __shared__ u32 s_w[kRgmThreads / 64];
    __shared__ int s_bnd[kMaxC][6];
    const int t = threadIdx.x, b = blockIdx.x;
    const RgView<NC> V = rg_view<NC>(a.cnt, a.map, Clouds{{a.app.p[0], a.app.p[1], a.app.p[2]}});
    int M = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) M += V.m[c];
    if (b == kRgmBuckets) {                            // (k_rgm_finish rewrites the counters after)
        finalize_pose(a.st, a.poses, a.pose_cap, 1, a.acc, a.st->params);
        return;
    }
    const RgmBox box = rgm_box(a.st->params);
    const int lo = rgm_bucket_lo<NC>(V, b), hi = rgm_bucket_lo<NC>(V, b + 1);
    RGM_MARK(0);
    const int nold = hi - lo;
    const bool cache = nold <= kRgmOldLds;
    // 1. this bucket's appended points (listed by the last LM launch), how many lie below it, and its
    // map points (keys, crop flags, still in key order?): all loads issued before any is waited on
    constexpr int kPerT = kRgmBucketCap / kRgmThreads;
    const int cnt_b = (int)a.bcount[b];
    int before = 0;
    for (int i = t; i < b; i += kRgmThreads) before += (int)a.bcount[i];
    const int c0 = min(cnt_b, kRgmBucketCap);
    u64 lk[kPerT];
    u32 lt[kPerT];
#pragma unroll
    for (int u = 0; u < kPerT; ++u) {
        const int i = t + u * kRgmThreads;
        if (i < c0) {
            lk[u] = a.bkey[(size_t)b * kRgmBucketCap + i];
            lt[u] = a.btag[(size_t)b * kRgmBucketCap + i];
        }
    }
    bool unsorted = false;
    for (int g = lo + t; g < hi; g += kRgmThreads) {
        int c, li;
        const int e = rgm_old_elem<NC>(V, g, c, li);
        const float4 p = a.map.at(c)[li];
        const u64 key = rgm_key(p, c, a.leaf.at(c), box);
        a.okey[g] = key;
        if (cache) {
            ok[g - lo] = key;
            opt[g - lo] = p;
        }
        a.key64[e] = key;
        a.vtag[e] = (u32)e | (box.in(p) ? 0u : kRgmDrop);
        if (g + 1 < M) unsorted |= rgm_old_key<NC>(V, a.leaf, box, g + 1) < key;
    }
    if (t == 0) {                              // the next bucket's splitter: the key of its first map point
        s_nextk = b + 1 < kRgmBuckets && hi < M ? rgm_old_key<NC>(V, a.leaf, box, hi) : ~0ull;
        s_cnt = cnt_b;
    }
    if (t < kMaxC) s_cls[t] = 0;
    rgm_bound_init(s_bnd, t);
    if (__any(unsorted) && lane_id() == 0) __hip_atomic_store(&a.stat[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int u = 0; u < kPerT; ++u) {
        const int i = t + u * kRgmThreads;
        if (i < c0) {
            bk[i] = lk[u];
            bt[i] = lt[u];
        }
    }
    before = wave_sum_i(before);
    if (lane_id() == 0) s_before[t >> 6] = before;
    __syncthreads();
    RGM_MARK(1);
    int nbefore = 0;
#pragma unroll
    for (int w = 0; w < kRgmThreads / 64; ++w) nbefore += s_before[w];
    const bool overflow = s_cnt > kRgmBucketCap;       // too many: the fallback sorts (still take part below)
    const int cb = overflow ? 0 : s_cnt;
    RGM_MARK(2);
    if (a.dbg && t == 0) a.dbg[64 + 10 * b + 9] = (unsigned long long)s_cnt;
    if (overflow && t == 0) __hip_atomic_store(&a.stat[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // 3. sort the bucket's appended points by (key, element)
    if (cb <= kRgmThreads) {
        // rank by counting: every element against every other through LDS broadcast reads (no
        // dependent stages; the typical bucket holds a few dozen appended points)
        const u64 k = t < cb ? bk[t] : ~0ull;
        const u32 g = t < cb ? bt[t] : ~0u;
        int rank = 0;
        if (t < cb)
            for (int j = 0; j < cb; ++j) rank += rgm_less(bk[j], bt[j], k, g) ? 1 : 0;
        __syncthreads();
        if (t < cb) {
            bk[rank] = k;
            bt[rank] = g;
        }
    } else if (cb <= 2 * kRgmThreads) rgm_sort_regs<2>(bk, bt, cb);
    else if (cb <= 4 * kRgmThreads) rgm_sort_regs<4>(bk, bt, cb);
    else rgm_sort_regs<8>(bk, bt, cb);
    __syncthreads();
    const bool acache = cb <= kRgmAppLds;              // the voxel walks then read LDS only
    if (acache)
        for (int r = t; r < cb; r += kRgmThreads) {
            int c;
            apt[r] = V.at((int)(bt[r] & ~kRgmDrop), c);
        }
    __syncthreads();
    RGM_MARK(3);
    // 4. voxels. Merged order: a map point after the appended points below it (equal keys: map points
    // first), an appended point after the map points at or below it. A voxel (a run of equal keys) is
    // reduced by the thread of its first element in this bucket: its map points in map order, then its
    // appended points; the voxel that opens the bucket may have map points in earlier buckets (equal
    // keys across a split), which leave it to this one. Every element writes its kept flag at its
    // merged position, a voxel's output sits at its first element's.
    const int L = nold + cb;
    const int base = lo + nbefore;
    const u64 s_next = s_nextk;
    auto okey_at = [&](int i) -> u64 { return cache ? ok[i] : a.okey[lo + i]; };
    auto add_old = [&](RgmVox& v, int g) {
        int c;
        const float4 p = cache && g >= lo ? opt[g - lo] : rgm_old_point<NC>(V, g, c);
        if (box.in(p)) v.add(p);
    };
    auto add_app = [&](RgmVox& v, int r) {            // sorted position r
        const u32 tag = bt[r];
        if (tag & kRgmDrop) return;
        int c;
        v.add(acache ? apt[r] : V.at((int)tag, c));
    };
    for (int i = t; i < nold; i += kRgmThreads) {
        const u64 K = okey_at(i);
        const int lb = rgm_lower(bk, cb, K);
        const int P = base + i + lb;
        u32 flag = 0;
        if ((i == 0 || okey_at(i - 1) != K) && (K < s_next || b == kRgmBuckets - 1)) {
            RgmVox v;
            if (i == 0) {                              // its map points in earlier buckets, in map order
                int g0 = lo;
                while (g0 > 0 && rgm_old_key<NC>(V, a.leaf, box, g0 - 1) == K) --g0;
                for (int g = g0; g < lo; ++g) add_old(v, g);
            }
            for (int j = i; j < nold && okey_at(j) == K; ++j) add_old(v, lo + j);
            for (int r = lb; r < cb && bk[r] == K; ++r) add_app(v, r);
            if (v.n) {
                float4 out;
                if (v.finish(a.k_new, a.theta_p, a.theta_max, out)) {
                    flag = 1u | (u32)(K >> 62) << 30;
                    atomicAdd(&s_cls[(int)(K >> 62)], 1);
                    rgm_bound_add(s_bnd, (int)(K >> 62), out);
                }
                a.vox[P] = out;
            }
        }
        a.kflag[P] = flag;
    }
    for (int r = t; r < cb; r += kRgmThreads) {
        const u64 K = bk[r];
        const int ub = cache ? rgm_upper(ok, nold, K) : rgm_upper(a.okey + lo, nold, K);
        const int P = base + r + ub;
        u32 flag = 0;
        if ((r == 0 || bk[r - 1] != K) && (ub == 0 || okey_at(ub - 1) != K)) {   // a voxel without map points
            RgmVox v;
            for (int q = r; q < cb && bk[q] == K; ++q) add_app(v, q);
            if (v.n) {
                float4 out;
                if (v.finish(a.k_new, a.theta_p, a.theta_max, out)) {
                    flag = 1u | (u32)(K >> 62) << 30;
                    atomicAdd(&s_cls[(int)(K >> 62)], 1);
                    rgm_bound_add(s_bnd, (int)(K >> 62), out);
                }
                a.vox[P] = out;
            }
        }
        a.kflag[P] = flag;
    }
    __syncthreads();
    RGM_MARK(4);
    // 5. the kept voxels' ranks in merged order, and the bucket's numbers for k_rgm_finish (which places
    // them in the other map set once every bucket is done: no workgroup waits on another here, so any
    // number of handles may run this kernel at once)
    u32 run = 0;
    for (int t0 = 0; t0 < L; t0 += kRgmThreads) {
        const int p = t0 + t;
        const u32 fl = p < L ? a.kflag[base + p] : 0u;
        const u32 f = fl & 0x3FFFFFFFu ? 1u : 0u;
        u32 tot;
        const u32 ex = block_excl_scan1024(f, s_w, tot);
        if (f) a.kflag[base + p] = (fl & 0xC0000000u) | (run + ex + 1);
        run += tot;
    }
    RGM_MARK(5);
    int* m = a.bmeta + kRgmMeta * b;
    if (t == 0) {
        m[0] = base;
        m[1] = L;
#pragma unroll
        for (int c = 0; c < kMaxC; ++c) m[2 + c] = c < NC ? s_cls[c] : 0;
    }
    if (t < 6 * NC) m[kRgmBnd + t] = s_bnd[t / 6][t % 6];
}

constexpr int kFbThreads = 256;

// Fallback: one 256-thread workgroup (a cheap launch when it has nothing to do) sorts all n (key64, vtag) pairs of element order stably by
// key into (kout, vout): LSD radix over 8-bit digits, passes whose digit is the same for every key
// skipped; tiles of 1024 keys ranked as in k_os_pass (a wave's 256 keys by match_bits, wave offsets
// by one barrier), one running digit base instead of a look-back.
__device__ void rgm_fallback_sort(const RgmArgs& a, int n) {
    __shared__ u32 hist[8][256];
    __shared__ u32 wcnt[kFbThreads / 64][256];
    __shared__ u32 gbase[256], toff[256];
    __shared__ int s_one[8];
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    for (int i = t; i < 8 * 256; i += kFbThreads) (&hist[0][0])[i] = 0;
    if (t < 8) s_one[t] = 0;
    __syncthreads();
    for (int i = t; i < n; i += kFbThreads) {
        const u64 k = a.key64[i];
#pragma unroll
        for (int p = 0; p < 8; ++p) atomicAdd(&hist[p][(u32)(k >> (8 * p)) & 255u], 1u);
    }
    __syncthreads();
    for (int i = t; i < 8 * 256; i += kFbThreads)
        if ((&hist[0][0])[i] == (u32)n) s_one[i >> 8] = 1;       // a digit the same for every key
    __syncthreads();
    u32 active = 0;                                    // digits that vary, as a bit mask
    int P = 0;
    for (int p = 0; p < 8; ++p)
        if (!s_one[p]) {
            active |= 1u << p;
            ++P;
        }
    const u64* ks = a.key64;
    const u32* vs = a.vtag;
    if (P == 0) {
        for (int i = t; i < n; i += kFbThreads) {
            a.kout[i] = ks[i];
            a.vout[i] = vs[i];
        }
        __syncthreads();
        return;
    }
    u64* kd = (P & 1) ? a.kout : a.ktmp;
    u32* vd = (P & 1) ? a.vout : a.vtmp;
    for (int pi = 0; pi < P; ++pi) {
        const int p = __ffs(active) - 1;
        active &= active - 1;
        const int shift = 8 * p;
        if (t < 256) {                                 // exclusive digit bases
            u32 s = 0;
            for (int d = 0; d < t; ++d) s += hist[p][d];
            gbase[t] = s;
        }
        __syncthreads();
        for (int base = 0; base < n; base += kFbThreads * 4) {
            u64 key[4];
            u32 val[4], rk[4], dg[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = base + w * 256 + r * 64 + l;
                key[r] = i < n ? ks[i] : 0ull;
                val[r] = i < n ? vs[i] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) wcnt[w][l + 64 * k] = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool valid = base + w * 256 + r * 64 + l < n;
                const u32 d = (u32)(key[r] >> shift) & 255u;
                dg[r] = d;
                const u64 peers = match_bits(d, 8, valid);
                const u32 below = (u32)__popcll(peers & lt);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const u32 run = valid ? wcnt[w][d] : 0u;
                rk[r] = valid ? run + below : 0xFFFFFFFFu;
                if (valid && below == 0) wcnt[w][d] = run + (u32)__popcll(peers);
            }
            __syncthreads();
            if (t < 256) {
                u32 acc = 0;
                for (int ww = 0; ww < kFbThreads / 64; ++ww) {
                    const u32 c = wcnt[ww][t];
                    wcnt[ww][t] = acc;
                    acc += c;
                }
                toff[t] = gbase[t];
                gbase[t] += acc;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (rk[r] == 0xFFFFFFFFu) continue;
                const u32 pos = toff[dg[r]] + wcnt[w][dg[r]] + rk[r];
                kd[pos] = key[r];
                vd[pos] = val[r];
            }
            __syncthreads();
        }
        // this pass's global stores before the next pass reads them (one workgroup)
        __threadfence_block();
        __syncthreads();
        ks = kd;
        vs = vd;
        kd = (kd == a.kout) ? a.ktmp : a.kout;
        vd = (vd == a.vout) ? a.vtmp : a.vout;
    }
}

// Fallback, second half: the voxels of the sorted (kout, vout) reduced by the same workgroup, tile by
// tile in key order with a running count of kept voxels (cropped elements skipped; a voxel's first
// element is its first uncropped one); the kept voxels then go to the other map set at their
// class-map index, and the map sizes and class boundaries are written
template <int NC>
__device__ void rgm_fallback_tail(const RgmArgs& a, const RgView<NC>& V, int n) {
    __shared__ u32 s_w[kFbThreads / 64];
    __shared__ int s_cls[kMaxC];
    const int t = threadIdx.x;
    if (t < kMaxC) s_cls[t] = 0;
    __syncthreads();
    u32 run = 0;
    for (int t0 = 0; t0 < n; t0 += kFbThreads) {
        const int i = t0 + t;
        u32 flag = 0, cls = 0;
        float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < n && !(a.vout[i] & kRgmDrop)) {
            const u64 K = a.kout[i];
            bool first = true;
            for (int j = i - 1; j >= 0 && a.kout[j] == K; --j)
                if (!(a.vout[j] & kRgmDrop)) { first = false; break; }
            if (first) {
                RgmVox v;
                for (int e = i; e < n && a.kout[e] == K; ++e) {
                    const u32 tg = a.vout[e];
                    if (tg & kRgmDrop) continue;
                    int c;
                    v.add(V.at((int)tg, c));
                }
                if (v.finish(a.k_new, a.theta_p, a.theta_max, out)) {
                    flag = 1;
                    cls = (u32)(K >> 62);
                    atomicAdd(&s_cls[cls], 1);
                }
            }
        }
        u32 tot;
        const u32 ex = block_excl_scan256(flag, s_w, tot);
        if (flag) {                                    // by kept rank: the output and its class
            a.vox[run + ex] = out;
            a.kflag[run + ex] = cls;
        }
        run += tot;
    }
    __shared__ int s_bnd[kMaxC][6];
    rgm_bound_init(s_bnd, t);
    __threadfence_block();
    __syncthreads();
    int low[kMaxC + 1];
    low[0] = 0;
#pragma unroll
    for (int c = 1; c <= kMaxC; ++c) low[c] = low[c - 1] + s_cls[c - 1];
    bool over = false;
    for (u32 r = t; r < run; r += kFbThreads) {
        const int c = min((int)a.kflag[r], NC - 1);
        const u32 idx = r - (u32)low[c];
        const float4 v = a.vox[r];
        if (idx < a.map_cap) {
            a.mapw.at(c)[idx] = v;
            rgm_bound_add(s_bnd, c, v);
        } else {
            over = true;
        }
    }
    if (over) atomicOr(a.err_map, 1);
    __syncthreads();
    if (t == 0) {
        for (int c = 1; c <= kMaxC; ++c) a.cnt[C_NLT + c - 1] = low[c];
        int nloc[kGridMaps] = {0, 0, 0};
        for (int c = 0; c < NC; ++c) a.cnt[C_M + c] = nloc[c] = min(s_cls[c], (int)a.map_cap);
        a.cnt[C_KEEP_TOTAL] = low[kMaxC];
        a.cnt[C_NRG] = n;
        grid_dims(&s_bnd[0][0], nloc, a.gdims, a.gncells, a.gcell_cap, a.gerr);   // the next update's grid
    }
}

// The second half of the merge (one workgroup per bucket, after every bucket is done): bucket b's
// kept voxels go to their class-map index in the other map set (the class-c voxels of the buckets
// before it counted from their numbers); workgroup 0 also writes the map sizes, the class boundaries
// and the total. When the merge is void, workgroup 0 runs the fallback instead (a single-workgroup
// sort and reduction of every element) and the others only reset their bucket's list.
template <int NC>
__global__ void __launch_bounds__(kFbThreads) k_rgm_finish(RgmArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    __shared__ int s_red[kFbThreads / 64][kMaxC];
    __shared__ int s_red6[kFbThreads / 64][6 * kMaxC];
    __shared__ int s_pre[kMaxC], s_tot[kMaxC];
    const bool fb = a.stat[0] != 0;
    if (fb) {
        if (b != 0) {
            if (t == 0) a.bcount[b] = 0u;
            return;
        }
        const RgView<NC> V = rg_view<NC>(a.cnt, a.map, Clouds{{a.app.p[0], a.app.p[1], a.app.p[2]}});
        const int n = V.total();
        __syncthreads();                               // every thread has read the map sizes
        rgm_fallback_sort(a, n);
        __threadfence_block();
        __syncthreads();
        rgm_fallback_tail<NC>(a, V, n);
        if (t == 0) {
            a.bcount[0] = 0u;
            a.stat[1]++;
            const int A = n - (V.m[0] + (NC > 1 ? V.m[1] : 0) + (NC > 2 ? V.m[2] : 0));
            if (A > a.stat[2]) a.stat[2] = A;
            a.stat[0] = 0;
        }
        return;
    }
    // the kept class-c voxels of the buckets before b (and of all buckets, for workgroup 0)
    int pre[kMaxC] = {0, 0, 0}, all[kMaxC] = {0, 0, 0};
    for (int bb = t; bb < kRgmBuckets; bb += kFbThreads) {
        const int* m = a.bmeta + kRgmMeta * bb;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int v = m[2 + c];
            if (bb < b) pre[c] += v;
            all[c] += v;
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        pre[c] = wave_sum_i(pre[c]);
        all[c] = wave_sum_i(all[c]);
    }
    if (lane_id() == 0)
#pragma unroll
        for (int c = 0; c < NC; ++c) s_red[t >> 6][c] = pre[c];
    __syncthreads();
    if (t < NC) {
        int v = 0;
        for (int w = 0; w < kFbThreads / 64; ++w) v += s_red[w][t];
        s_pre[t] = v;
    }
    __syncthreads();
    if (lane_id() == 0)
#pragma unroll
        for (int c = 0; c < NC; ++c) s_red[t >> 6][c] = all[c];
    __syncthreads();
    if (t < NC) {
        int v = 0;
        for (int w = 0; w < kFbThreads / 64; ++w) v += s_red[w][t];
        s_tot[t] = v;
    }
    __syncthreads();
    const int* m = a.bmeta + kRgmMeta * b;
    const int base = m[0], L = m[1];
    u32 first_rank[kMaxC];                             // bucket-local rank of the first voxel of class c
    {
        u32 acc = 0;
#pragma unroll
        for (int c = 0; c < kMaxC; ++c) {
            first_rank[c] = acc;
            acc += c < NC ? (u32)m[2 + c] : 0u;
        }
    }
    bool over = false;
    for (int p = t; p < L; p += kFbThreads) {
        const u32 f = a.kflag[base + p];
        if (!(f & 0x3FFFFFFFu)) continue;
        const int c = min((int)(f >> 30), NC - 1);
        const u32 idx = (u32)sel3(c, s_pre[0], s_pre[1], s_pre[2]) + (f & 0x3FFFFFFFu) - 1u -
                        sel3(c, first_rank[0], first_rank[1], first_rank[2]);
        if (idx < a.map_cap) a.mapw.at(c)[idx] = a.vox[base + p];
        else over = true;
    }
    if (over) atomicOr(a.err_map, 1);
    __shared__ int s_bnd[kMaxC][6];
    if (b == 0) {                                      // the map grid's bounds: over every bucket's
        int v[6 * kMaxC];
#pragma unroll
        for (int k = 0; k < 6 * kMaxC; ++k) v[k] = (k % 6) < 3 ? INT_MAX : INT_MIN;
        for (int bb = t; bb < kRgmBuckets; bb += kFbThreads) {
            const int* mb = a.bmeta + kRgmMeta * bb + kRgmBnd;
#pragma unroll
            for (int k = 0; k < 6 * NC; ++k) v[k] = (k % 6) < 3 ? min(v[k], mb[k]) : max(v[k], mb[k]);
        }
#pragma unroll
        for (int k = 0; k < 6 * NC; ++k) {
            v[k] = (k % 6) < 3 ? wave_min_i(v[k]) : wave_max_i(v[k]);
            if (lane_id() == 0) s_red6[t >> 6][k] = v[k];
        }
        __syncthreads();
        if (t < 6 * kMaxC) {
            int r = (t % 6) < 3 ? INT_MAX : INT_MIN;
            if (t < 6 * NC)
                for (int w = 0; w < kFbThreads / 64; ++w) r = (t % 6) < 3 ? min(r, s_red6[w][t]) : max(r, s_red6[w][t]);
            s_bnd[t / 6][t % 6] = r;
        }
        __syncthreads();
    }
    if (t == 0) {
        a.bcount[b] = 0u;                              // the list of the next update
        if (b == 0) {
            const RgView<NC> V = rg_view<NC>(a.cnt, a.map, a.map);
            const int n = V.total();
            int M = 0;
            for (int c = 0; c < NC; ++c) M += V.m[c];
            int tot = 0;
            for (int c = 1; c <= kMaxC; ++c) {
                tot += c - 1 < NC ? s_tot[c - 1] : 0;
                a.cnt[C_NLT + c - 1] = tot;
            }
            int nloc[kGridMaps] = {0, 0, 0};
            for (int c = 0; c < NC; ++c) a.cnt[C_M + c] = nloc[c] = min(s_tot[c], (int)a.map_cap);
            a.cnt[C_KEEP_TOTAL] = tot;
            a.cnt[C_NRG] = n;
            if (n - M > a.stat[2]) a.stat[2] = n - M;
            grid_dims(&s_bnd[0][0], nloc, a.gdims, a.gncells, a.gcell_cap, a.gerr);   // the next update's grid
        }
    }
}

// initMapWithPoints (ES :217-222, BPF :685-691): append the raw clouds (r = g = 0)
template <int NC>
__global__ void __launch_bounds__(256) k_init_map(const int* __restrict__ cnt, Clouds in, CloudsW map) {
    const CatIdx<NC> ci = cat_idx<NC>(cnt + C_IN);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ci.total(); i += gridDim.x * blockDim.x) {
        const int c = ci.cls(i);
        const float4 p = in.at(c)[i - ci.start(c)];
        map.at(c)[cnt[C_M + c] + i - ci.start(c)] = make_float4(p.x, p.y, p.z, __uint_as_float(0u));
    }
}

// the maps (x, y, z, bits(r | g << 8)) and their sizes into mapped pinned host memory (PCIe writes)
__global__ void __launch_bounds__(256) k_map_export(const int* __restrict__ cnt, CloudsW map, CloudsW out,
                                                     int* __restrict__ out_n, int nc) {
    for (int c = 0; c < nc; ++c) {
        const int n = cnt[C_M + c];
        if (blockIdx.x == 0 && threadIdx.x == 0) out_n[c] = n;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
            out.at(c)[i] = map.at(c)[i];
    }
}

__global__ void k_init_buckets(int4* __restrict__ b, size_t n) {   // n buckets
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * kBktQuads; i += (size_t)gridDim.x * blockDim.x)
        b[i] = (i % kBktQuads) == 0 ? make_int4(0, -1, -1, -1) : make_int4(-1, -1, -1, -1);
}

__global__ void k_init_counts(int* __restrict__ cnt, DevState* __restrict__ st, int nc) {
    if (threadIdx.x != 0) return;
    for (int c = 0; c < nc; ++c) cnt[C_M + c] += cnt[C_IN + c];
    st->optimization_count = 12;
}

}  // namespace

// ==============================================================================================
// (Re)create stage A's stream, restricted to all but the last `reserve` CUs (0: unrestricted).
// A reserve that would leave stage A fewer than 32 CUs is PF_EINVAL. The new stream is created
// before the old one is destroyed, so a failure leaves the handle's stage A stream valid. The masked
// stream is a blocking stream (hipExtStreamCreateWithCUMask takes no flags), so the C ABI keeps every
// copy stream-ordered on the handle's streams and never uses the null stream.
int odom_masked_stream(int device, int reserve, hipStream_t* out) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return PF_EHIP;
    if (reserve < 0 || (reserve > 0 && reserve > ncu - 32)) return PF_EINVAL;
    hipStream_t s = nullptr;
    if (reserve > 0) {
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int c = 0; c < ncu - reserve; ++c) mask[c / 32] |= 1u << (c % 32);
        if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) return PF_EHIP;
    } else if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        return PF_EHIP;
    }
    *out = s;
    return PF_OK;
}

hipError_t odom_sync_a(OdomGPU& o) {
    for (hipStream_t f : o.stream_f)
        if (f) {
            const hipError_t e = hipStreamSynchronize(f);
            if (e != hipSuccess) return e;
        }
    return o.stream_a ? hipStreamSynchronize(o.stream_a) : hipSuccess;
}

int odom_stage_a_stream(OdomGPU& o, int reserve) {
    if (odom_sync_a(o) != hipSuccess) return PF_EHIP;
    hipStream_t s = nullptr, f[2] = {};
    if (int rc = odom_masked_stream(o.device, reserve, &s)) return rc;
    for (int l = 0; l < 2; ++l)                        // the front-end lanes share stage A's CUs
        if (o.stream_f[l])
            if (int rc = odom_masked_stream(o.device, reserve, &f[l])) {
                (void)hipStreamDestroy(s);
                if (f[0]) (void)hipStreamDestroy(f[0]);
                return rc;
            }
    if (o.stream_a) (void)hipStreamDestroy(o.stream_a);
    o.stream_a = s;
    for (int l = 0; l < 2; ++l)
        if (o.stream_f[l]) {
            (void)hipStreamDestroy(o.stream_f[l]);
            o.stream_f[l] = f[l];
        }
    o.cu_reserve = reserve;
    // graphs were captured on the old stream's work; they are stream-independent, keep them
    return PF_OK;
}

void alias_err(int*& flag, int* word) {
    if (flag != word) (void)hipFree(flag);
    flag = word;
}

// development: PF_TRACE_CREATE=1 prints the create steps (stderr)
static void trace_create(const char* step) {
    static const bool on = std::getenv("PF_TRACE_CREATE") != nullptr;
    if (on) std::fprintf(stderr, "pf create: %s\n", step);
}

int odom_create(OdomGPU& o, const pf_lidar_params& lidar, const pf_odom_params& prm, int device, size_t in_cap,
                size_t map_cap, int nc) {
    if (nc < 2 || nc > kMaxC) return PF_EINVAL;
    trace_create("begin");
    o.lidar = lidar;
    o.prm = prm;
    o.device = device;
    o.in_cap = in_cap;
    o.map_cap = map_cap;
    o.cls = ClassCfg{nc, 1u << (nc - 1)};          // the last class is the plane class
    o.sort_cap = (size_t)nc * (map_cap + in_cap);
    if (o.sort_cap < 10 * in_cap) o.sort_cap = 10 * in_cap;
    o.pose_cap = (size_t)1 << 20;
    for (int c = 0; c < nc; ++c) {
        const bool plane = o.cls.is_plane(c);
        o.leaf_vg[c] = plane ? (float)(prm.map_res * 2) : (float)prm.map_res;   // setLeafSize(double -> float)
        o.leaf_rg[c] = plane ? (float)prm.map_res * 2 : (float)prm.map_res;     // float map_resolution (.h:62)
    }
    if (hipStreamCreateWithFlags(&o.stream, hipStreamNonBlocking) != hipSuccess) return PF_EHIP;
    if (hipStreamCreateWithFlags(&o.stream_bx, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&o.ev_bx_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&o.ev_bx_join, hipEventDisableTiming) != hipSuccess)
        return PF_EHIP;
    if (const char* e = std::getenv("PF_TIE_AUX")) o.tie_aux = std::atoi(e) != 0;   // development A/B
    if (const char* e = std::getenv("PF_TIE_HS")) o.tie_hs = std::atoi(e) != 0;
    trace_create("stream");
    // stage A is kept off the last compute units by default (odom_stage_a_stream), so that stage B's
    // kernels — the LM needs kLmBlocks co-resident workgroups — find free CUs while stage A runs
    int reserve = nc == 2 ? kStageAReserveES : kStageAReserveBPF;
    if (const char* e = std::getenv("PF_STAGE_A_CU_RESERVE")) reserve = std::atoi(e);   // development override
    if (odom_stage_a_stream(o, reserve) != PF_OK && odom_stage_a_stream(o, 0) != PF_OK) return PF_EHIP;
    trace_create("stage A stream");
    if (std::getenv("PF_STAGE_B_CU_EXCL") && reserve > 0) {   // development: stage B on the reserved CUs only
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, o.device) != hipSuccess) return PF_EHIP;
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int c = ncu - reserve; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
        hipStream_t sb = nullptr;
        if (hipExtStreamCreateWithCUMask(&sb, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
            (void)hipStreamDestroy(o.stream);
            o.stream = sb;
        }
    }
    int rc = fe_alloc(o.fe, lidar, in_cap);
    if (rc) return rc;
    trace_create("fe_alloc");
    // 1 m cells over every map's bounding box: 3 x (201 m)^2 x 270 m covers the +-100 m crop box
    rc = grid_alloc(o.grid, (size_t)nc * map_cap, (size_t)1 << 25);
    if (rc) return rc;
    rc = prim_alloc(o.prim, o.sort_cap, ((size_t)1 << 25) + 2);   // sorts; scans up to the cell count
    if (rc) return rc;
    rc = prim_alloc(o.vprim, (size_t)nc * in_cap);
    if (rc) return rc;
    trace_create("grid / prims");
    const size_t nq = (size_t)nc * in_cap;
#define PF_ALLOC(ptr, bytes) \
    if (hipMalloc(&(ptr), (bytes)) != hipSuccess) return PF_ENOMEM;
    PF_ALLOC(o.st, sizeof(DevState));
    PF_ALLOC(o.lm, sizeof(LMState));
    PF_ALLOC(o.cnt, sizeof(int) * C_COUNT);
    PF_ALLOC(o.acc, sizeof(u32) * A_COUNT);
    for (int p = 0; p < kSlots; ++p) {
        for (int c = 0; c < nc; ++c) {
            PF_ALLOC(o.sb[p].in[c], sizeof(float4) * in_cap);
            PF_ALLOC(o.sb[p].ds[c], sizeof(float4) * in_cap);
        }
        PF_ALLOC(o.sb[p].cnt, sizeof(int) * C_COUNT);
        if (hipMemsetAsync(o.sb[p].cnt, 0, sizeof(int) * C_COUNT, o.stream) != hipSuccess) return PF_EHIP;
        if (hipEventCreateWithFlags(&o.ev_a[p], hipEventDisableTiming) != hipSuccess) return PF_EHIP;
        if (hipEventCreateWithFlags(&o.ev_b[p], hipEventDisableTiming) != hipSuccess) return PF_EHIP;
    }
    PF_ALLOC(o.acc_a, sizeof(u32) * A_COUNT);
    PF_ALLOC(o.vkeys, sizeof(u32) * (nq + 1));
    PF_ALLOC(o.vvals, sizeof(u32) * (nq + 1));
    PF_ALLOC(o.vflags, sizeof(u32) * (nq + 1));
    PF_ALLOC(o.vscan, sizeof(u32) * (nq + 1));
    PF_ALLOC(o.vsegstart, sizeof(u32) * (nq + 1));
    for (int c = 0; c < nc; ++c) {
        PF_ALLOC(o.mapset[0][c], sizeof(float4) * map_cap);
        PF_ALLOC(o.mapset[1][c], sizeof(float4) * map_cap);
        PF_ALLOC(o.app[c], sizeof(float4) * in_cap);
    }
    PF_ALLOC(o.seg_out, sizeof(float4) * o.sort_cap);
    o.tail_tiles = (o.sort_cap + kTailTile - 1) / kTailTile;
    PF_ALLOC(o.tail_status, sizeof(u64) * (o.tail_tiles + 1));    // look-back words + the arrival counter
    PF_ALLOC(o.keys, sizeof(u32) * (o.sort_cap + 1));
    PF_ALLOC(o.vals, sizeof(u32) * (o.sort_cap + 1));
    PF_ALLOC(o.nbr, sizeof(int) * 5 * nq);
    PF_ALLOC(o.qflag, sizeof(int) * nq);
    PF_ALLOC(o.lm_part, sizeof(double) * kLmEvals * kLmBlocks * 32);
    PF_ALLOC(o.lm_ticket, sizeof(u32) * 2 * kLmEvalSlots);
    PF_ALLOC(o.errw, sizeof(int) * E_COUNT);
    PF_ALLOC(o.geo, sizeof(double) * 8 * nq);
    PF_ALLOC(o.spars, sizeof(float) * nq);
    PF_ALLOC(o.roundv, sizeof(float) * nq);
    PF_ALLOC(o.observe, sizeof(float) * nq);
    PF_ALLOC(o.pnext, sizeof(int) * 5 * nq);
    PF_ALLOC(o.pbkt, sizeof(int4) * kBktQuads * nc * map_cap);
    PF_ALLOC(o.tailinc, sizeof(u32) * 5 * nq);
    PF_ALLOC(o.poses, sizeof(double) * 7 * o.pose_cap);
    PF_ALLOC(o.stage, sizeof(float4) * nq);
    PF_ALLOC(o.rgm_okey, sizeof(u64) * nc * map_cap);
    PF_ALLOC(o.rgm_key64, sizeof(u64) * o.sort_cap);
    PF_ALLOC(o.rgm_vtag, sizeof(u32) * o.sort_cap);
    PF_ALLOC(o.rgm_kout, sizeof(u64) * o.sort_cap);
    PF_ALLOC(o.rgm_ktmp, sizeof(u64) * o.sort_cap);
    PF_ALLOC(o.rgm_vtmp, sizeof(u32) * o.sort_cap);
    PF_ALLOC(o.rgm_bcount, sizeof(u32) * kRgmBuckets);
    PF_ALLOC(o.rgm_bmeta, sizeof(int) * kRgmMeta * kRgmBuckets);
    PF_ALLOC(o.dims_next, sizeof(int) * (8 * kGridMaps + 1));
    PF_ALLOC(o.rgm_bkey, sizeof(u64) * kRgmBuckets * kRgmBucketCap);
    PF_ALLOC(o.rgm_btag, sizeof(u32) * kRgmBuckets * kRgmBucketCap);
    PF_ALLOC(o.rgm_vox, sizeof(float4) * o.sort_cap);
    PF_ALLOC(o.rgm_kflag, sizeof(u32) * o.sort_cap);
    PF_ALLOC(o.rgm_stat, sizeof(int) * 8);
#undef PF_ALLOC
    trace_create("buffers");
    if (std::getenv("PF_PROBE")) {                 // development probe: LM phase timestamps
        if (hipMalloc(&o.dbg, sizeof(unsigned long long) * kDbgWords) != hipSuccess) return PF_ENOMEM;
        if (hipMemset(o.dbg, 0, sizeof(unsigned long long) * kDbgWords) != hipSuccess) return PF_EHIP;
    }
    if (hipHostMalloc(&o.h_cnt, sizeof(int) * (C_COUNT + E_COUNT)) != hipSuccess) return PF_ENOMEM;   // + errw mirror
    if (hipHostMalloc(&o.h_pose, sizeof(double) * 8) != hipSuccess) return PF_ENOMEM;
    if (hipHostMalloc(&o.h_rd, sizeof(HostRead), hipHostMallocMapped) != hipSuccess) return PF_ENOMEM;
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&o.h_rd_dev), o.h_rd, 0) != hipSuccess) return PF_EHIP;
    // init (:182-208, BPF :649-681): identity odom / last_odom, parameters {0,0,0,1,0,0,0},
    // optimization_count 2
    DevState h{};
    h.params[3] = 1.0;
    for (int i = 0; i < 3; ++i) h.odomR[4 * i] = h.lastR[4 * i] = 1.0;
    h.optimization_count = 2;
    trace_create("pinned");
    // stream-ordered on the handle's own non-blocking stream (null-stream copies would also wait for
    // every blocking stream of the process, e.g. other handles' CU-masked stage-A streams)
    if (hipMemcpyAsync(o.st, &h, sizeof(h), hipMemcpyHostToDevice, o.stream) != hipSuccess) return PF_EHIP;
    trace_create("state copy");
    if (hipMemsetAsync(o.cnt, 0, sizeof(int) * C_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.acc, 0, sizeof(u32) * A_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.acc_a, 0, sizeof(u32) * A_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.lm, 0, sizeof(LMState), o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.lm_ticket, 0, sizeof(u32) * 2 * kLmEvalSlots, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.errw, 0, sizeof(int) * E_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.tail_status, 0, sizeof(u64) * (o.tail_tiles + 1), o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.rgm_stat, 0, sizeof(int) * 8, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.rgm_bcount, 0, sizeof(u32) * kRgmBuckets, o.stream) != hipSuccess) return PF_EHIP;
    // the sub-objects' overflow / wait flags latch into the handle's sticky error words
    alias_err(o.fe.err, o.errw + E_FE_SECTOR);
    alias_err(o.grid.err, o.errw + E_GRID);
    alias_err(o.prim.err, o.errw + E_SORT_B);
    alias_err(o.vprim.err, o.errw + E_SORT_A);
    trace_create("memsets");
    hipLaunchKernelGGL(k_init_buckets, dim3(1024), dim3(256), 0, o.stream, o.pbkt, (size_t)nc * map_cap);   // all empty
    if (hipStreamSynchronize(o.stream) != hipSuccess) return PF_EHIP;
    trace_create("done");
    o.opt_count_host = 2;
    return PF_OK;
}

// back to the state after init (identity pose, empty maps, optimization_count 2), keeping every
// allocation and captured graph: the next frame seeds the maps again
__global__ void k_dep_dirty(u32* dirty) {
    if (threadIdx.x == 0) {
        dirty[0] = 1u;
        dirty[1] = 0u;
    }
}

// the maps were written other than by the tie-order rgbds: the next one takes the full table (DepTab)
void odom_dep_dirty(OdomGPU& o, hipStream_t s) {
    if (o.dep_dirty) hipLaunchKernelGGL(k_dep_dirty, dim3(1), dim3(64), 0, s, o.dep_dirty);
}

// the table holds every element of one rgbds call (at most sort_cap) at a load of at most 0.8, and never
// fewer than the 2^kDepSmallBits slots the small-table path (dep_small, k_rg_dep_probe, k_rg_dep) hashes
// into and scans whatever the handle's capacity
int odom_dep_alloc(OdomGPU& o) {
    if (o.dep_key) return PF_OK;
    u32 hb = kDepSmallBits;
    while (((size_t)1 << hb) < o.sort_cap + o.sort_cap / 4) ++hb;
    const size_t h = (size_t)1 << hb;
    int rc = PF_OK;
    if (hipMalloc(&o.dep_key, sizeof(u32) * h) != hipSuccess || hipMalloc(&o.dep_cnt, sizeof(u32) * h) != hipSuccess ||
        hipMalloc(&o.dep_mem, sizeof(u32) * 3 * h) != hipSuccess ||
        hipMalloc(&o.dep_slot, sizeof(u32) * o.sort_cap) != hipSuccess ||
        hipMalloc(&o.dep_free, o.sort_cap) != hipSuccess || hipMalloc(&o.dep_dirty, sizeof(u32) * 2) != hipSuccess) {
        rc = PF_ENOMEM;
    } else {
        const u32 dirty0[2] = {1u, 0u};
        if (hipMemset(o.dep_key, 0xFF, sizeof(u32) * h) != hipSuccess ||
            hipMemset(o.dep_cnt, 0, sizeof(u32) * h) != hipSuccess ||
            hipMemcpy(o.dep_dirty, dirty0, sizeof(dirty0), hipMemcpyHostToDevice) != hipSuccess)
            rc = PF_EHIP;
    }
    if (rc != PF_OK) {                 // nothing half-allocated stays behind (a later call retries cleanly)
        odom_dep_release(o);
        return rc;
    }
    o.dep_hbits = hb;
    return PF_OK;
}

void odom_dep_release(OdomGPU& o) {
    for (void* q : {(void*)o.dep_key, (void*)o.dep_cnt, (void*)o.dep_mem, (void*)o.dep_slot, (void*)o.dep_free,
                    (void*)o.dep_dirty})
        if (q) (void)hipFree(q);
    o.dep_key = o.dep_cnt = o.dep_mem = o.dep_slot = o.dep_dirty = nullptr;
    o.dep_free = nullptr;
    o.dep_hbits = 0;
}

int odom_reset(OdomGPU& o) {
    if (odom_sync_a(o) != hipSuccess || hipStreamSynchronize(o.stream) != hipSuccess) return PF_EHIP;
    DevState h{};
    h.params[3] = 1.0;
    for (int i = 0; i < 3; ++i) h.odomR[4 * i] = h.lastR[4 * i] = 1.0;
    h.optimization_count = 2;
    if (hipMemcpyAsync(o.st, &h, sizeof(h), hipMemcpyHostToDevice, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.cnt, 0, sizeof(int) * C_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.acc, 0, sizeof(u32) * A_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.acc_a, 0, sizeof(u32) * A_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.lm, 0, sizeof(LMState), o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.lm_ticket, 0, sizeof(u32) * 2 * kLmEvalSlots, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.errw, 0, sizeof(int) * E_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.tail_status, 0, sizeof(u64) * (o.tail_tiles + 1), o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.rgm_stat, 0, sizeof(int) * 8, o.stream) != hipSuccess) return PF_EHIP;
    if (hipMemsetAsync(o.rgm_bcount, 0, sizeof(u32) * kRgmBuckets, o.stream) != hipSuccess) return PF_EHIP;
    for (int p = 0; p < kSlots; ++p)
        if (hipMemsetAsync(o.sb[p].cnt, 0, sizeof(int) * C_COUNT, o.stream) != hipSuccess) return PF_EHIP;
    hipLaunchKernelGGL(k_init_buckets, dim3(1024), dim3(256), 0, o.stream, o.pbkt, (size_t)o.cls.nc * o.map_cap);
    if (o.front && o.front->dcvc && dcvc_reset(*o.front->dcvc, o.stream) != PF_OK) return PF_EHIP;   // a first frame again
    if (o.front2 && o.front2->dcvc && dcvc_mark_called(*o.front2->dcvc, o.stream) != PF_OK) return PF_EHIP;
    if (hipStreamSynchronize(o.stream) != hipSuccess) return PF_EHIP;
    o.dcvc_first = o.front && o.front->dcvc;
    o.tie_hint = 0;
    o.opt_count_host = 2;
    o.inited = false;
    o.dims_fresh = false;
    o.frames = 0;
    o.err_seen = 0;
    o.rd_frames = -1;
    return PF_OK;
}

void odom_destroy(OdomGPU& o) {
    for (int p = 0; p < kSlots; ++p) {
        if (o.graph_a[p]) (void)hipGraphExecDestroy(o.graph_a[p]);
        for (int q = 0; q < 2; ++q)
            if (o.graph_b[p + kSlots * q]) (void)hipGraphExecDestroy(o.graph_b[p + kSlots * q]);
        if (o.graph_as[p]) (void)hipGraphExecDestroy(o.graph_as[p]);
        for (int l = 0; l < 2; ++l)
            if (o.graph_f[p + kSlots * l]) (void)hipGraphExecDestroy(o.graph_f[p + kSlots * l]);
        if (o.ev_f[p]) (void)hipEventDestroy(o.ev_f[p]);
        if (o.ev_a[p]) (void)hipEventDestroy(o.ev_a[p]);
        if (o.ev_b[p]) (void)hipEventDestroy(o.ev_b[p]);
        for (int c = 0; c < kMaxC; ++c) {
            (void)hipFree(o.sb[p].in[c]);
            (void)hipFree(o.sb[p].ds[c]);
        }
        (void)hipFree(o.sb[p].cnt);
    }
    // aliased flags point into errw (freed below), not at their own allocations
    if (o.errw) {
        o.fe.err = nullptr;
        o.grid.err = nullptr;
        o.prim.err = nullptr;
        o.vprim.err = nullptr;
        if (o.front) o.front->grid.err = nullptr;
        if (o.front2) o.front2->grid.err = nullptr;
    }
    fe_free(o.fe);
    for (ClsGPU* f : {o.front, o.front2})
        if (f) {
            cls_free(*f);
            delete f;
        }
    (void)hipFree(o.stage2);
    for (hipStream_t f : o.stream_f)
        if (f) (void)hipStreamDestroy(f);
    grid_free(o.grid);
    prim_free(o.prim);
    prim_free(o.vprim);
    for (int c = 0; c < kMaxC; ++c) {
        for (int q = 0; q < 2; ++q) (void)hipFree(o.mapset[q][c]);
        (void)hipFree(o.app[c]);
    }
    void* ptrs[] = {o.st, o.lm, o.cnt, o.acc, o.acc_a, o.vkeys, o.vvals, o.vflags, o.vscan, o.vsegstart, o.seg_out,
                    o.keys, o.vals, o.tail_status, o.nbr, o.qflag, o.lm_part, o.lm_ticket, o.geo,
                    o.spars, o.roundv, o.observe, o.pnext, o.pbkt, o.tailinc, o.poses, o.stage, o.dbg, o.errw,
                    o.rgm_okey, o.rgm_key64, o.rgm_vtag, o.rgm_kout, o.rgm_ktmp, o.rgm_vox, o.rgm_kflag, o.rgm_bcount, o.rgm_bmeta, o.rgm_bkey,
                    o.rgm_btag, o.rgm_vtmp, o.rgm_stat, o.dims_next};
    for (void* q : ptrs) (void)hipFree(q);
    if (o.h_cnt) (void)hipHostFree(o.h_cnt);
    if (o.h_pose) (void)hipHostFree(o.h_pose);
    if (o.h_rd) (void)hipHostFree(o.h_rd);
    if (o.hs) {
        for (int p = 0; p < kSlots; ++p) {
            if (o.hs->h[p]) (void)hipHostFree(o.hs->h[p]);
            (void)hipFree(o.hs->d[p]);
            if (o.hs->ev[p]) (void)hipEventDestroy(o.hs->ev[p]);
        }
        if (o.hs->stream) (void)hipStreamDestroy(o.hs->stream);
        delete o.hs;
    }
    for (int c = 0; c < kMaxC; ++c)
        if (o.h_map[c]) (void)hipHostFree(o.h_map[c]);
    if (o.h_map_n) (void)hipHostFree(o.h_map_n);
    if (o.stream) (void)hipStreamDestroy(o.stream);
    if (o.stream_a) (void)hipStreamDestroy(o.stream_a);
    if (o.stream_bx) (void)hipStreamDestroy(o.stream_bx);
    if (o.ev_bx_fork) (void)hipEventDestroy(o.ev_bx_fork);
    if (o.ev_bx_join) (void)hipEventDestroy(o.ev_bx_join);
    for (TieSort* t : {o.tie_a, o.tie_b})
        if (t) {
            tie_free(*t);
            delete t;
        }
    odom_dep_release(o);
    o = OdomGPU{};
}

static Clouds clouds(float4* const* p) { return Clouds{{p[0], p[1], p[2]}}; }

// kernels specialised on the class count (2: ES, 3: BPF)
#define PF_LAUNCH_NC(nc, kern, ...)                                   \
    do {                                                              \
        if ((nc) == 3) hipLaunchKernelGGL(kern<3>, __VA_ARGS__);      \
        else hipLaunchKernelGGL(kern<2>, __VA_ARGS__);                \
    } while (0)
static CloudsW clouds_w(float4* const* p) { return CloudsW{{p[0], p[1], p[2]}}; }

void stage_enqueue_fe(OdomGPU& o, int p, const float4* d_in, hipStream_t s) {
    StageBuf& sb = o.sb[p];
    fe_enqueue(o.fe, d_in, sb.cnt + C_NIN, sb.in[0], sb.cnt + C_IN, sb.in[1], sb.cnt + C_IN + 1, s);
}

void stage_enqueue_vg(OdomGPU& o, int p, hipStream_t s) {
    StageBuf& sb = o.sb[p];
    int* cnt = sb.cnt;
    const int nc = o.cls.nc;
    const VgLeaf leaf{{o.leaf_vg[0], o.leaf_vg[1], o.leaf_vg[2]}};
    // VoxelGrid of every class (:242-245, BPF :714-719); pose independent, so it runs ahead on stream A
    hipLaunchKernelGGL(k_vg_begin, dim3(1), dim3(64), 0, s, cnt, o.acc_a, nc);
    PF_LAUNCH_NC(nc, k_vg_minmax, dim3(128), dim3(256), 0, s, clouds(sb.in), cnt, o.acc_a);
    PF_LAUNCH_NC(nc, k_vg_keys, dim3(kGrid), dim3(256), 0, s, clouds(sb.in), cnt, o.acc_a, leaf, o.vkeys, o.vvals,
                 sort_hist(o.vprim, 32, true));
    if (o.tie_order)                       // std::sort's order of equal keys (PCL VoxelGrid, B.1)
        tie_sort(*o.tie_a, o.vkeys, o.vvals, TieClasses{cnt, C_IN, -1, nc}, o.vprim.err, s, PF_TIE_LEVELS_A);
    else
        radix_sort_pairs(o.vkeys, o.vvals, cnt + C_VGN, 32, o.vprim, s, nullptr, nullptr, true);
    segment_starts(o.vkeys, cnt + C_VGN, o.vsegstart, cnt + C_NSEG, cnt + C_NLT, cnt + C_NRG_VALID, o.vprim, s);
    PF_LAUNCH_NC(nc, k_vg_reduce, dim3(kGrid * 4), dim3(256), 0, s, clouds(sb.in), o.vkeys, o.vvals, o.vsegstart, cnt,
                 clouds_w(sb.ds));
}

void odom_enqueue_export(OdomGPU& o, hipStream_t s, bool after_update) {
    if (!o.export_maps) return;
    hipLaunchKernelGGL(k_map_export, dim3(256), dim3(256), 0, s, o.cnt,
                       clouds_w(after_update ? map_next(o) : map_cur(o)), clouds_w(o.h_map_dev),
                       o.h_map_n_dev, o.cls.nc);
}

void odom_enqueue_init(OdomGPU& o, int p, hipStream_t s) {
    StageBuf& sb = o.sb[p];
    const int nc = o.cls.nc;
    hipLaunchKernelGGL(k_pull_counts, dim3(1), dim3(64), 0, s, o.cnt, sb.cnt);
    PF_LAUNCH_NC(nc, k_init_map, dim3(kGrid), dim3(256), 0, s, o.cnt, clouds(sb.in), clouds_w(map_cur(o)));
    odom_dep_dirty(o, s);                                // initMapWithPoints: several points per voxel
    hipLaunchKernelGGL(k_init_counts, dim3(1), dim3(64), 0, s, o.cnt, o.st, nc);
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, o.st, o.poses, (int)o.pose_cap, 0, o.acc);
    o.opt_count_host = 12;
    o.inited = true;
    o.dims_fresh = false;
}

#ifndef PF_ODOM_GRID_AGG
#define PF_ODOM_GRID_AGG 0      // development A/B: 1 = one counter atomic per run of equal cells in a wave
#endif
void odom_enqueue_update(OdomGPU& o, int p, hipStream_t s) {
    if (o.opt_count_host > 2) o.opt_count_host--;
    StageBuf& sb = o.sb[p];
    int* cnt = o.cnt;
    const int nc = o.cls.nc;
    // (a side-stream branch for the single-thread prediction beside the grid build measured slower
    // under graph replay: 2815 vs 2930 frames/s; the fork / join edges cost more than the overlap;
    // as the tail of the bounds kernel it overlaps for free)
    // grids of the class maps (kd-tree builds, :249-250 / BPF :723-725); the pose prediction rides on
    // the bounds kernel as its tail (it reads the map sizes of the previous frame, not the grid)
    GridPtrs gp{{map_cur(o)[0], map_cur(o)[1], map_cur(o)[2]}, {cnt + C_M, cnt + C_M + 1, cnt + C_M + 2}, nc};
    const PredictTail pred{o.st, cnt, sb.cnt, o.acc, o.cls};
    if (o.dims_fresh) {                       // dims from the previous update's k_rgm_finish: the count first
        hipLaunchKernelGGL((k_grid_count<PF_ODOM_GRID_AGG != 0, FreshTail>), dim3(kGridCountBlocks + 1), dim3(256), 0, s, gp,
                           o.dims_next, o.grid.cell_count, o.grid.slot, o.grid.ttot, o.grid.err,
                           FreshTail{pred, o.dims_next, o.grid.dims, o.grid.d_ncells});
        grid_scan_scatter(o.grid, gp, s);
    } else {
        hipLaunchKernelGGL(k_grid_bounds<PredictTail>, dim3(kGridBoundsBlocks + 1), dim3(256), 0, s,
                           grid_bounds_args(o.grid, gp), pred);
        grid_build(o.grid, gp, o.prim, s, true, PF_ODOM_GRID_AGG != 0);
    }
    // (PF_ODOM_GRID_AGG, round 6: the count's atomics taken per run of equal cells in a wave, as the front
    // end's: measured slightly slower here, configs[4] 315 vs 317 and the headline 912 vs 915 frames/s --
    // voxel order at the 0.4 / 0.8 m leaves gives short runs of 1 m cells -- so one atomic per point stays)
    const GridView gv{o.grid.dims, o.grid.cell_start, o.grid.cpts};
    for (int it = 0; it < o.opt_count_host; ++it) {
        AssocArgs aa{o.st, cnt, o.acc, gv, o.cls, clouds(sb.ds), clouds(map_cur(o)), o.nbr, o.qflag, o.geo, o.spars,
                     o.roundv, o.pbkt, o.pnext, (u32)o.map_cap, o.lm_ticket, o.lm_part};
        PF_LAUNCH_NC(nc, k_assoc, dim3(kGrid), dim3(256), 0, s, aa);
        ObsArgs oa{cnt, o.acc, o.cls, clouds(map_cur(o)), clouds_w(sb.ds), o.nbr, o.qflag, o.pbkt, o.pnext, o.tailinc,
                   (u32)o.map_cap, o.roundv, o.spars, o.observe, o.prm.k_new, o.prm.theta_p, o.prm.theta_max,
                   o.errw + E_LM};
        // weightType 0 needs no frame-wide observe / sparsity bounds before the solve: the observe pass
        // runs inside k_lm_solve, chunk by chunk, and k_observe is not launched
        const bool fuse = o.prm.weight_type == 0 && !o.no_fuse_obs;
        if (!fuse) PF_LAUNCH_NC(nc, k_observe, dim3(kGrid), dim3(256), 0, s, oa);
        const bool merge = !o.tie_order && !o.rg_radix;
        const RgmPrep prep{merge && it == o.opt_count_host - 1, clouds(map_cur(o)), clouds(sb.ds), clouds_w(o.app),
                           o.rgm_key64, o.rgm_vtag, VgLeaf{{o.leaf_rg[0], o.leaf_rg[1], o.leaf_rg[2]}}, o.rgm_bcount,
                           o.rgm_bkey, o.rgm_btag, o.rgm_stat};
        LmArgs la{o.st, cnt, o.acc, o.cls, o.lm, o.lm_part, o.lm_ticket, o.qflag, clouds(sb.ds), o.geo, o.observe,
                  o.spars, o.prm.weight_type, o.dbg, o.nbr, o.tailinc, o.pbkt, clouds_w(map_cur(o)), (u32)o.map_cap,
                  o.errw + E_LM, prep, oa, fuse ? 1 : 0};
        PF_LAUNCH_NC(nc, k_lm_solve, dim3(kLmBlocks), dim3(256), 0, s, la);   // grid must be kLmBlocks
    }
    // pose (:278-280, node copy.cpp:105-107) and addPointsToMap (:589-647, BPF :1197-1290)
    const VgLeaf leaf{{o.leaf_rg[0], o.leaf_rg[1], o.leaf_rg[2]}};
    if (!o.tie_order && !o.rg_radix) {                    // rgbds by merge (the map stays in key order)
        RgmArgs ra{o.st, cnt, o.acc, clouds(map_cur(o)), clouds(sb.ds), clouds_w(o.app), o.poses, (int)o.pose_cap,
                   leaf, o.prm.k_new, o.prm.theta_p, o.prm.theta_max, o.rgm_okey, o.rgm_key64, o.rgm_vtag,
                   o.rgm_vox, o.rgm_kflag, clouds_w(map_next(o)), (u32)o.map_cap, o.errw + E_MAP, o.rgm_kout, o.vals, o.rgm_ktmp, o.rgm_vtmp,
                   o.rgm_stat, o.rgm_bmeta, o.dims_next, o.dims_next + 8 * kGridMaps, (long long)o.grid.cell_cap,
                   o.grid.err,
                   o.rgm_bcount, o.rgm_bkey, o.rgm_btag, o.dbg};
        PF_LAUNCH_NC(nc, k_rgm_bucket, dim3(kRgmBuckets + 1), dim3(kRgmThreads), 0, s, ra);
        PF_LAUNCH_NC(nc, k_rgm_finish, dim3(kRgmBuckets), dim3(kFbThreads), 0, s, ra);
        o.dims_fresh = true;
        return;
    }
    o.dims_fresh = false;
    // the order-free voxel groups (the heap tier's dependence flags) in the tie order
    const DepTab dt{o.tie_order ? o.dep_key : nullptr, o.dep_cnt, o.dep_mem, o.dep_slot, o.dep_free, o.dep_hbits,
                    o.dep_dirty};
    if (dt.key && o.dep_force_full) odom_dep_dirty(o, s);   // test switch: the full table every update
    if (rg_fused_keys(o.leaf_rg, nc)) {
        PF_LAUNCH_NC(nc, k_rg_append_keys, dim3(kGrid + 1), dim3(256), 0, s, o.st, cnt, o.acc, clouds(map_cur(o)),
                     clouds(sb.ds), clouds_w(o.app), o.poses, (int)o.pose_cap, leaf, o.keys, o.vals,
                     sort_hist(o.prim, 32, true), dt);
    } else {
        PF_LAUNCH_NC(nc, k_rg_append_minmax, dim3(256 + 1), dim3(256), 0, s, o.st, cnt, o.acc, clouds(map_cur(o)),
                     clouds(sb.ds), clouds_w(o.app), o.poses, (int)o.pose_cap);
        PF_LAUNCH_NC(nc, k_rg_keys, dim3(kGrid), dim3(256), 0, s, o.st, cnt, o.acc, clouds(map_cur(o)), clouds(o.app),
                     leaf, o.keys, o.vals, sort_hist(o.prim, 32, true), dt);
    }
    if (o.tie_order) {                     // std::sort's order of equal keys (:74)
        if (dt.key) {
            PF_LAUNCH_NC(nc, k_rg_dep_probe, dim3(kGrid), dim3(256), 0, s, cnt, o.keys, dt);
            PF_LAUNCH_NC(nc, k_rg_dep, dim3(kGrid), dim3(256), 0, s, cnt, clouds(map_cur(o)), clouds(o.app), dt);
        }
        TieAux aux;
        aux.s = o.tie_aux ? o.stream_bx : nullptr;
        aux.fork = o.ev_bx_fork;
        aux.join = o.ev_bx_join;
        // the side-stream radix route only for eager launches: captured into stage B's graph (several
        // handles, PF_GRAPH_AUTO) the fork / join measured slower than the route on the stage's own stream
        // (configs[4] 173 against 281 frames/s in the full bench), so a captured stage B keeps it in line
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        (void)hipStreamIsCapturing(s, &cap);
        aux.hs = o.tie_hs && cap == hipStreamCaptureStatusNone ? o.stream_bx : nullptr;
        tie_sort(*o.tie_b, o.keys, o.vals, TieClasses{cnt, C_M, C_DS, nc}, o.prim.err, s,
                 std::max(tie_levels_for(*o.tie_b, o.tie_hint), PF_TIE_LEVELS_B), dt.key ? o.dep_free : nullptr,
                 &aux);
    }
    else
        radix_sort_pairs(o.keys, o.vals, cnt + C_NRG, 32, o.prim, s, nullptr, nullptr, true);
    u32* dirty = o.tie_order ? o.dep_dirty : nullptr;
    RgTailArgs ta{cnt, clouds(map_cur(o)), clouds(o.app), o.keys, o.vals, o.seg_out, o.prm.k_new, o.prm.theta_p,
                  o.prm.theta_max, o.tail_status, (u32*)(o.tail_status + o.tail_tiles), o.prim.err, leaf, dirty};
    const unsigned tail_grid = (unsigned)(o.tail_tiles < (size_t)kSortMaxBlocks ? o.tail_tiles : kSortMaxBlocks);
    PF_LAUNCH_NC(nc, k_rg_tail, dim3(tail_grid > 0 ? tail_grid : 1), dim3(256), 0, s, ta);
    PF_LAUNCH_NC(nc, k_rg_write, dim3(kGrid), dim3(256), 0, s, cnt, o.seg_out, clouds_w(map_next(o)), dirty);
}

// the association kNN probe (pf_odom.h)
int odom_probe_assoc(OdomGPU& o, int iters, double* avg_ms, double* alg_bytes, int* nq_out, float4* q_host,
                     size_t q_cap) {
    if (!o.inited || o.frames < 2 || iters < 1) return PF_EINVAL;
    const int nc = o.cls.nc;
    const int p = (o.frames - 1) % kSlots;
    int nq = 0;
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    PF_HIP_TRY(hipMemcpy(&nq, o.cnt + C_NQ, sizeof(int), hipMemcpyDeviceToHost));
    *nq_out = nq;
    if (nq <= 0) return PF_EINVAL;
    int* nbr = nullptr;
    float4* qd = nullptr;
    unsigned long long* bytes = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = PF_OK;
    if (hipMalloc(&nbr, sizeof(int) * (size_t)nq) != hipSuccess || hipMalloc(&qd, sizeof(float4) * (size_t)nq) != hipSuccess ||
        hipMalloc(&bytes, sizeof(unsigned long long)) != hipSuccess)
        rc = PF_ENOMEM;
    if (!rc && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) rc = PF_EHIP;
    const GridView gv{o.grid.dims, o.grid.cell_start, o.grid.cpts};
    const Clouds ds = clouds(o.sb[p].ds);
    if (!rc) {
        auto launch = [&](float4* qo) {
            if (nq <= kAssocWideMax) PF_LAUNCH_NC(nc, k_assoc_probe_t16, dim3(kGrid), dim3(256), 0, o.stream, o.st, o.cnt, gv, ds, nbr, qo);
            else PF_LAUNCH_NC(nc, k_assoc_probe_t8, dim3(kGrid), dim3(256), 0, o.stream, o.st, o.cnt, gv, ds, nbr, qo);
        };
        launch(qd);                                   // warm-up, and the queries for the caller
        (void)hipMemsetAsync(bytes, 0, sizeof(unsigned long long), o.stream);
        PF_LAUNCH_NC(nc, k_assoc_cellpop, dim3(kGrid), dim3(256), 0, o.stream, o.st, o.cnt, gv, ds, bytes);
        (void)hipEventRecord(e0, o.stream);
        for (int i = 0; i < iters; ++i) launch(nullptr);
        (void)hipEventRecord(e1, o.stream);
        float ms = 0.f;
        unsigned long long b = 0;
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess ||
            hipMemcpy(&b, bytes, sizeof(b), hipMemcpyDeviceToHost) != hipSuccess)
            rc = PF_EHIP;
        *avg_ms = (double)ms / iters;
        *alg_bytes = (double)b;
        if (!rc && q_host && q_cap >= (size_t)nq &&
            hipMemcpy(q_host, qd, sizeof(float4) * (size_t)nq, hipMemcpyDeviceToHost) != hipSuccess)
            rc = PF_EHIP;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(nbr);
    (void)hipFree(qd);
    (void)hipFree(bytes);
    return rc;
}

}  // namespace pf
