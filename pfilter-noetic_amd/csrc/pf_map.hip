// LaserMappingClass (src/laserMappingClass.cpp) on the device: the global map of 50 m cubes.
//
// The map is one array of points (x, y, z, intensity) with the global cube coordinates of each
// point; inside a cube the points keep the reference's order (the last VoxelGrid output in ascending
// voxel index, then later additions in push order). One updateCurrentPointsToMap (:151-189) is
//   k_map_transform   scan -> world (PCL's f32 Transformer order), intensity from the sensor z,
//                     cube of every point; points outside the 5x5x5 neighbourhood are counted
//   k_map_bounds      per neighbourhood cube (125): min / max of its points (ordered-int atomics)
//   k_map_dims        per cube: PCL VoxelGrid's min_b / divisions (B.1)
//   k_map_keys        sort key per point: 0 outside the neighbourhood (kept as they are), else
//                     1 << 31 | cube << 24 | voxel index
//   radix sort (stable) -> k_map_flags + scan -> k_map_reduce: every voxel's centroid (sequential
//                     f32 sums in sorted = reference order), every kept point copied
// and getMap (:194-206) is a stable sort of the array by global cube (x, then y, then z).
#include "pf_common.h"
#include "pf_prims.h"

#include <cfloat>
#include <climits>
#include <cmath>
#include <mutex>
#include <set>
#include <tuple>
#include <vector>

namespace pf {
namespace {

constexpr double kCell = 50.0;     // LASER_CELL_WIDTH / HEIGHT / DEPTH (include/laserMappingClass.h:13-15)
constexpr int kRange = 2;          // LASER_CELL_RANGE_HORIZONTAL / VERTICAL (:19-20)
constexpr int kSide = 2 * kRange + 1;
constexpr int kCubes = kSide * kSide * kSide;
constexpr int kCubeBias = 512;     // global cube coordinates packed as 3 x 10 bits
constexpr u32 kVoxelBits = 24;

__device__ __forceinline__ int cube_of(double v) { return (int)floor(v / kCell + 0.5); }
__device__ __forceinline__ u32 pack_cube(int x, int y, int z) {
    return ((u32)(x + kCubeBias) << 20) | ((u32)(y + kCubeBias) << 10) | (u32)(z + kCubeBias);
}
__device__ __forceinline__ int unpack(u32 k, int sh) { return (int)((k >> sh) & 1023u) - kCubeBias; }

struct MapDev {
    float4* pts;          // [cap] current map (first *n_map), then this update's points
    u32* cube;            // [cap] packed global cube per point
    int* cnt;             // [8]: 0 map size, 1 new points, 2 outside the neighbourhood, 3 kept (key 0),
                          //      4 error (cube grid too fine), 5 outside the cube-coordinate range
    u32* bounds;          // [kCubes * 6] ordered-float min x, y, z, max x, y, z
    int* dims;            // [kCubes * 6] min_b x, y, z, div x, div x*y, valid
    u32* keys;
    u32* vals;
    u32* flags;
    u32* scan;
    float4* out;          // [cap] next map
    u32* out_cube;
    float leaf;
    int cx, cy, cz;       // the current position's cube
};

__device__ __forceinline__ int local_cube(const MapDev& d, u32 k) {
    const int x = unpack(k, 20) - d.cx + kRange, y = unpack(k, 10) - d.cy + kRange, z = unpack(k, 0) - d.cz + kRange;
    if (x < 0 || x >= kSide || y < 0 || y >= kSide || z < 0 || z >= kSide) return -1;
    return (x * kSide + y) * kSide + z;
}

// the scan to world: pcl::transformPointCloud with pose.cast<float>() (PCL 1.10 Transformer<float>::se3:
// x c0 + (y c1 + (z c2 + c3))), intensity = min(1, max(z + 2, 0) / 5) in double (:167), cube (:168-170)
__global__ void __launch_bounds__(256) k_map_transform(const float4* __restrict__ scan, int n, MapDev d,
                                                       float c00, float c01, float c02, float c10, float c11,
                                                       float c12, float c20, float c21, float c22, float t0,
                                                       float t1, float t2) {
    const int m = d.cnt[0];
    int outside = 0, range = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = scan[i];
        const float x = p.x * c00 + (p.y * c10 + (p.z * c20 + t0));
        const float y = p.x * c01 + (p.y * c11 + (p.z * c21 + t1));
        const float z = p.x * c02 + (p.y * c12 + (p.z * c22 + t2));
        const float in = (float)fmin(1.0, fmax((double)p.z + 2.0, 0.0) / 5);
        const int gx = cube_of((double)x), gy = cube_of((double)y), gz = cube_of((double)z);
        const bool ok = gx > -kCubeBias && gx < kCubeBias && gy > -kCubeBias && gy < kCubeBias && gz > -kCubeBias &&
                        gz < kCubeBias;
        range += !ok;
        const u32 k = ok ? pack_cube(gx, gy, gz) : 0u;
        outside += ok && local_cube(d, k) < 0;
        d.pts[m + i] = make_float4(x, y, z, in);
        d.cube[m + i] = k;
    }
    outside = wave_sum_i(outside);
    range = wave_sum_i(range);
    if (lane_id() == 0) {
        if (outside) atomicAdd(&d.cnt[2], outside);
        if (range) atomicAdd(&d.cnt[5], range);
    }
}

// per-cube bounds: LDS atomics per workgroup (points of a frame crowd into a few cubes; global
// atomics on 6 x 125 words serialised at ~4 ms), then one global atomic per touched word
__global__ void __launch_bounds__(256) k_map_bounds(MapDev d) {
    __shared__ u32 lb[kCubes * 6];
    for (int k = threadIdx.x; k < kCubes * 6; k += blockDim.x) lb[k] = (k % 6) < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    const int tot = d.cnt[0] + d.cnt[1];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
        const int lc = local_cube(d, d.cube[i]);
        if (lc < 0) continue;
        const float4 p = d.pts[i];
        u32* b = lb + 6 * lc;
        atomicMin(&b[0], f2ord(p.x)); atomicMin(&b[1], f2ord(p.y)); atomicMin(&b[2], f2ord(p.z));
        atomicMax(&b[3], f2ord(p.x)); atomicMax(&b[4], f2ord(p.y)); atomicMax(&b[5], f2ord(p.z));
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kCubes * 6; k += blockDim.x) {
        const u32 v = lb[k];
        if ((k % 6) < 3) {
            if (v != 0xFFFFFFFFu) atomicMin(&d.bounds[k], v);
        } else if (v != 0u) {
            atomicMax(&d.bounds[k], v);
        }
    }
}

// PCL VoxelGrid (B.1) per cube: min_b = floor(min * inv), divisions, and the overflow guard
__global__ void k_map_dims(MapDev d) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= kCubes) return;
    u32* b = d.bounds + 6 * c;
    int* o = d.dims + 6 * c;
    const float inv = 1.0f / d.leaf;
    const float mn[3] = {ord2f(b[0]), ord2f(b[1]), ord2f(b[2])}, mx[3] = {ord2f(b[3]), ord2f(b[4]), ord2f(b[5])};
    o[5] = 0;
    if (mn[0] <= mx[0]) {                           // the cube has points
        const long long ex = (long long)((mx[0] - mn[0]) * inv) + 1, ey = (long long)((mx[1] - mn[1]) * inv) + 1,
                        ez = (long long)((mx[2] - mn[2]) * inv) + 1;
        int mb[3], db[3];
        for (int k = 0; k < 3; ++k) {
            mb[k] = (int)floorf(mn[k] * inv);
            db[k] = (int)floorf(mx[k] * inv) - mb[k] + 1;
        }
        const long long nv = (long long)db[0] * db[1] * db[2];
        if (ex * ey * ez > (long long)INT_MAX) {
            // PCL: "leaf size too small", the cube is left as it is (key 0 below)
        } else if (nv > (1ll << kVoxelBits)) {
            atomicOr(&d.cnt[4], 1);                 // beyond the sort key's voxel field
        } else {
            o[0] = mb[0]; o[1] = mb[1]; o[2] = mb[2]; o[3] = db[0]; o[4] = db[0] * db[1]; o[5] = 1;
        }
    }
    b[0] = b[1] = b[2] = 0xFFFFFFFFu;               // reset for the next update
    b[3] = b[4] = b[5] = 0u;
}

__global__ void __launch_bounds__(256) k_map_keys(MapDev d) {
    __shared__ int kept;
    if (threadIdx.x == 0) kept = 0;
    __syncthreads();
    const int tot = d.cnt[0] + d.cnt[1];
    const float inv = 1.0f / d.leaf;
    int mine = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
        const int lc = local_cube(d, d.cube[i]);
        u32 key = 0;
        if (lc >= 0 && d.dims[6 * lc + 5]) {
            const int* o = d.dims + 6 * lc;
            const float4 p = d.pts[i];
            const int i0 = (int)(floorf(p.x * inv) - (float)o[0]);
            const int i1 = (int)(floorf(p.y * inv) - (float)o[1]);
            const int i2 = (int)(floorf(p.z * inv) - (float)o[2]);
            key = (1u << 31) | ((u32)lc << kVoxelBits) | (u32)(i0 + i1 * o[3] + i2 * o[4]);
        }
        mine += key == 0;
        d.keys[i] = key;
        d.vals[i] = (u32)i;
    }
    mine = wave_sum_i(mine);
    if (lane_id() == 0 && mine) atomicAdd(&kept, mine);
    __syncthreads();
    if (threadIdx.x == 0 && kept) atomicAdd(&d.cnt[3], kept);
}

// output slots: every kept point, and the first point of every voxel run
__global__ void __launch_bounds__(256) k_map_flags(MapDev d, const u32* __restrict__ ks) {
    const int tot = d.cnt[0] + d.cnt[1];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x)
        d.flags[i] = (ks[i] == 0u || i == 0 || ks[i] != ks[i - 1]) ? 1u : 0u;
}

__global__ void __launch_bounds__(256) k_map_reduce(MapDev d, const u32* __restrict__ ks, const u32* __restrict__ vs) {
    const int tot = d.cnt[0] + d.cnt[1];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
        if (!d.flags[i]) continue;
        const u32 k = ks[i];
        const u32 o = d.scan[i];
        if (k == 0u) {
            d.out[o] = d.pts[vs[i]];
            d.out_cube[o] = d.cube[vs[i]];
            continue;
        }
        float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
        int j = i;
        for (; j < tot && ks[j] == k; ++j) {
            const float4 p = d.pts[vs[j]];
            sx += p.x; sy += p.y; sz += p.z; si += p.w;
        }
        const float n = (float)(j - i);
        d.out[o] = make_float4(sx / n, sy / n, sz / n, si / n);
        d.out_cube[o] = d.cube[vs[i]];
    }
}

__global__ void k_map_commit(MapDev d, const u32* __restrict__ scan_total) {
    d.cnt[0] = (int)*scan_total;
    d.cnt[1] = 0;
}

// getMap: sort key = the packed global cube (x, then y, then z), stable
__global__ void __launch_bounds__(256) k_map_order(MapDev d) {
    const int m = d.cnt[0];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        d.keys[i] = d.cube[i];
        d.vals[i] = (u32)i;
    }
}
__global__ void __launch_bounds__(256) k_map_gather(MapDev d, const u32* __restrict__ vs, float4* __restrict__ out) {
    const int m = d.cnt[0];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[i] = d.pts[vs[i]];
}

}  // namespace
}  // namespace pf

using namespace pf;

struct pf_map {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t cap = 0, scan_cap = 0;
    float leaf = 0.4f;
    MapDev d{};
    float4* scan_buf = nullptr;     // staging of host scans
    PrimWork w;
    int* h_cnt = nullptr;           // pinned [8]
    std::set<std::tuple<int, int, int>> allocated;   // cubes the reference has allocated (init, checkPoints)
    std::vector<float4> host;
};

namespace {
void map_free(pf_map* h) {
    void* ps[] = {h->d.pts, h->d.cube, h->d.cnt, h->d.bounds, h->d.dims, h->d.keys, h->d.vals, h->d.flags,
                  h->d.scan, h->d.out, h->d.out_cube, h->scan_buf};
    for (void* p : ps) (void)hipFree(p);
    prim_free(h->w);
    if (h->h_cnt) (void)hipHostFree(h->h_cnt);
    if (h->stream) (void)hipStreamDestroy(h->stream);
}

void allocate_around(pf_map* h, int cx, int cy, int cz) {     // init (:7-33) / checkPoints (:136-146)
    for (int i = cx - kRange; i <= cx + kRange; ++i)
        for (int j = cy - kRange; j <= cy + kRange; ++j)
            for (int k = cz - kRange; k <= cz + kRange; ++k) h->allocated.insert(std::make_tuple(i, j, k));
}

int cube_host(double v) { return (int)std::floor(v / kCell + 0.5); }

// the node's pose: Isometry3d::Identity().rotate(Quaterniond(w, x, y, z)).pretranslate(t)
// (src/laserMappingNode.cpp:78-80); Eigen's toRotationMatrix
void pose_to_T(const double p[7], double T[12]) {
    const double x = p[0], y = p[1], z = p[2], w = p[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x,
                 txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
    const double R[3][3] = {{1 - (tyy + tzz), txy - twz, txz + twy},
                            {txy + twz, 1 - (txx + tzz), tyz - twx},
                            {txz - twy, tyz + twx, 1 - (txx + tyy)}};
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T[4 * r + c] = R[r][c];
        T[4 * r + 3] = p[4 + r];
    }
}

// T: row-major [R | t] (3 x 4) of the Isometry3d the node builds
int map_update(pf_map* h, const float4* d_scan, size_t n, const double T[12]) {
    MapDev& d = h->d;
    PF_HIP_TRY(hipSetDevice(h->device));
    if (n > h->scan_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    if ((size_t)h->h_cnt[0] + n > h->cap) return PF_ECAPACITY;
    const double R[3][3] = {{T[0], T[1], T[2]}, {T[4], T[5], T[6]}, {T[8], T[9], T[10]}};
    const double pose[7] = {0, 0, 0, 1, T[3], T[7], T[11]};
    d.cx = cube_host(pose[4]);
    d.cy = cube_host(pose[5]);
    d.cz = cube_host(pose[6]);
    allocate_around(h, d.cx, d.cy, d.cz);
    const int ni = (int)n;
    PF_HIP_TRY(hipMemsetAsync(d.cnt + 1, 0, sizeof(int) * 7, h->stream));
    PF_HIP_TRY(hipMemcpyAsync(d.cnt + 1, &ni, sizeof(int), hipMemcpyHostToDevice, h->stream));
    if (n)
        hipLaunchKernelGGL(k_map_transform, dim3(256), dim3(256), 0, h->stream, d_scan, ni, d, (float)R[0][0],
                           (float)R[1][0], (float)R[2][0], (float)R[0][1], (float)R[1][1], (float)R[2][1],
                           (float)R[0][2], (float)R[1][2], (float)R[2][2], (float)pose[4], (float)pose[5],
                           (float)pose[6]);
    PF_HIP_TRY(hipMemcpyAsync(h->h_cnt, d.cnt, sizeof(int) * 8, hipMemcpyDeviceToHost, h->stream));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    if (h->h_cnt[5]) return PF_EINVAL;                        // beyond +-25 km of the origin
    if (h->h_cnt[2]) {
        // points outside the neighbourhood: the reference pushes them into their cube if it was ever
        // allocated, else dereferences a null cloud (checked here before the map changes)
        std::vector<u32> cubes(n);
        PF_HIP_TRY(hipMemcpy(cubes.data(), d.cube + h->h_cnt[0], sizeof(u32) * n, hipMemcpyDeviceToHost));
        for (u32 k : cubes) {
            const auto c = std::make_tuple((int)((k >> 20) & 1023u) - kCubeBias, (int)((k >> 10) & 1023u) - kCubeBias,
                                           (int)(k & 1023u) - kCubeBias);
            if (!h->allocated.count(c)) return PF_EINVAL;
        }
    }
    hipLaunchKernelGGL(k_map_bounds, dim3(512), dim3(256), 0, h->stream, d);
    hipLaunchKernelGGL(k_map_dims, dim3(1), dim3(128), 0, h->stream, d);
    hipLaunchKernelGGL(k_map_keys, dim3(512), dim3(256), 0, h->stream, d);
    // sort over the map plus the new points: the count lives at cnt[0] + cnt[1]; stage it at cnt[6]
    const int tot = h->h_cnt[0] + ni;
    PF_HIP_TRY(hipMemcpyAsync(d.cnt + 6, &tot, sizeof(int), hipMemcpyHostToDevice, h->stream));
    u32 *ks = nullptr, *vs = nullptr;
    radix_sort_pairs(d.keys, d.vals, d.cnt + 6, 32, h->w, h->stream, &ks, &vs);
    hipLaunchKernelGGL(k_map_flags, dim3(512), dim3(256), 0, h->stream, d, ks);
    scan_exclusive(d.flags, d.scan, d.cnt + 6, reinterpret_cast<u32*>(d.cnt + 7), h->w, h->stream);
    hipLaunchKernelGGL(k_map_reduce, dim3(512), dim3(256), 0, h->stream, d, ks, vs);
    hipLaunchKernelGGL(k_map_commit, dim3(1), dim3(1), 0, h->stream, d, reinterpret_cast<const u32*>(d.cnt + 7));
    std::swap(d.pts, d.out);
    std::swap(d.cube, d.out_cube);
    PF_HIP_TRY(hipMemcpyAsync(h->h_cnt, d.cnt, sizeof(int) * 8, hipMemcpyDeviceToHost, h->stream));
    PF_HIP_TRY(hipGetLastError());
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    return h->h_cnt[4] ? PF_EUNSUPPORTED : PF_OK;             // a cube's voxel lattice above 2^24 cells
}
}  // namespace

extern "C" {

int pf_map_create(double map_resolution, int device, size_t max_points, size_t max_scan, pf_map** out) {
    if (!out || !(map_resolution > 0.0) || max_points == 0 || max_scan == 0 || max_points + max_scan > (size_t)INT_MAX)
        return PF_EINVAL;
    *out = nullptr;
    int ndev = 0;
    PF_HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(device));
    pf_map* h = new pf_map();
    h->device = device;
    h->cap = max_points + max_scan;
    h->scan_cap = max_scan;
    h->leaf = (float)map_resolution;                           // setLeafSize(float, float, float)
    h->d.leaf = h->leaf;
    const size_t c = h->cap;
    int rc = PF_OK;
#define PF_MAP_ALLOC(p, bytes) \
    if (rc == PF_OK && hipMalloc(&(p), (bytes)) != hipSuccess) rc = PF_ENOMEM
    PF_MAP_ALLOC(h->d.pts, sizeof(float4) * c);
    PF_MAP_ALLOC(h->d.out, sizeof(float4) * c);
    PF_MAP_ALLOC(h->d.cube, sizeof(u32) * c);
    PF_MAP_ALLOC(h->d.out_cube, sizeof(u32) * c);
    PF_MAP_ALLOC(h->d.keys, sizeof(u32) * c);
    PF_MAP_ALLOC(h->d.vals, sizeof(u32) * c);
    PF_MAP_ALLOC(h->d.flags, sizeof(u32) * c);
    PF_MAP_ALLOC(h->d.scan, sizeof(u32) * c);
    PF_MAP_ALLOC(h->d.cnt, sizeof(int) * 8);
    PF_MAP_ALLOC(h->d.bounds, sizeof(u32) * 6 * kCubes);
    PF_MAP_ALLOC(h->d.dims, sizeof(int) * 6 * kCubes);
    PF_MAP_ALLOC(h->scan_buf, sizeof(float4) * max_scan);
#undef PF_MAP_ALLOC
    if (rc == PF_OK && hipHostMalloc(&h->h_cnt, sizeof(int) * 8) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) rc = PF_EHIP;
    if (rc == PF_OK) rc = prim_alloc(h->w, c);
    if (rc == PF_OK) {
        std::vector<u32> b(6 * kCubes);
        for (int k = 0; k < kCubes; ++k)
            for (int j = 0; j < 6; ++j) b[6 * k + j] = j < 3 ? 0xFFFFFFFFu : 0u;
        if (hipMemcpy(h->d.bounds, b.data(), sizeof(u32) * b.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemset(h->d.cnt, 0, sizeof(int) * 8) != hipSuccess)
            rc = PF_EHIP;
        std::fill(h->h_cnt, h->h_cnt + 8, 0);
    }
    if (rc != PF_OK) {
        map_free(h);
        delete h;
        return rc;
    }
    allocate_around(h, 0, 0, 0);
    *out = h;
    return PF_OK;
}

int pf_map_destroy(pf_map* h) {
    if (!h) return PF_EINVAL;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    map_free(h);
    delete h;
    return PF_OK;
}

int pf_map_update(pf_map* h, const float* xyzi, size_t n, size_t stride_bytes, const double pose[7]) {
    if (!h || !pose || (!xyzi && n) || stride_bytes < 12) return PF_EINVAL;
    if (n > h->scan_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(h->device));
    h->host.resize(n);
    const char* b = reinterpret_cast<const char*>(xyzi);
    for (size_t i = 0; i < n; ++i) {
        const float* p = reinterpret_cast<const float*>(b + i * stride_bytes);
        h->host[i] = make_float4(p[0], p[1], p[2], stride_bytes >= 16 ? p[3] : 0.f);
    }
    if (n) PF_HIP_TRY(hipMemcpyAsync(h->scan_buf, h->host.data(), sizeof(float4) * n, hipMemcpyHostToDevice, h->stream));
    double T[12];
    pose_to_T(pose, T);
    return map_update(h, h->scan_buf, n, T);
}

int pf_map_update_mat(pf_map* h, const float* xyzi, size_t n, size_t stride_bytes, const double T[12]) {
    if (!h || !T || (!xyzi && n) || stride_bytes < 12) return PF_EINVAL;
    if (n > h->scan_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(h->device));
    h->host.resize(n);
    const char* b = reinterpret_cast<const char*>(xyzi);
    for (size_t i = 0; i < n; ++i) {
        const float* p = reinterpret_cast<const float*>(b + i * stride_bytes);
        h->host[i] = make_float4(p[0], p[1], p[2], stride_bytes >= 16 ? p[3] : 0.f);
    }
    if (n) PF_HIP_TRY(hipMemcpyAsync(h->scan_buf, h->host.data(), sizeof(float4) * n, hipMemcpyHostToDevice, h->stream));
    return map_update(h, h->scan_buf, n, T);
}

int pf_map_update_device(pf_map* h, const float* d_xyzi, size_t n, const double pose[7]) {
    if (!h || !pose || (!d_xyzi && n)) return PF_EINVAL;
    double T[12];
    pose_to_T(pose, T);
    return map_update(h, reinterpret_cast<const float4*>(d_xyzi), n, T);
}

int pf_map_get(pf_map* h, float* xyzi, size_t cap, size_t* n) {
    if (!h || !n) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->device));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    const size_t m = (size_t)h->h_cnt[0];
    *n = m;
    if (!xyzi) return PF_OK;
    if (m > cap) return PF_ECAPACITY;
    if (!m) return PF_OK;
    MapDev& d = h->d;
    hipLaunchKernelGGL(k_map_order, dim3(512), dim3(256), 0, h->stream, d);
    u32 *ks = nullptr, *vs = nullptr;
    radix_sort_pairs(d.keys, d.vals, d.cnt, 30, h->w, h->stream, &ks, &vs);
    hipLaunchKernelGGL(k_map_gather, dim3(512), dim3(256), 0, h->stream, d, vs, d.out);
    PF_HIP_TRY(hipMemcpyAsync(xyzi, d.out, sizeof(float4) * m, hipMemcpyDeviceToHost, h->stream));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    return PF_OK;
}

}  // extern "C"
