// C ABI (include/pfilter_hip.h) over the device pipeline. Host code here only stages inputs,
// enqueues work on the handle's stream and copies results back; all arithmetic is on the device.
#include <algorithm>
#include <chrono>
#include <climits>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "pf_fe.h"
#include "pf_odom.h"
#include "pf_geom.h"

using namespace pf;

namespace {

__global__ void k_set_int(int* p, int v) {
    if (threadIdx.x == 0) *p = v;
}
__global__ void k_set_counts(int* p, int a, int b, int c, int nc) {
    const int t = threadIdx.x;
    if (t < nc) p[t] = t == 0 ? a : (t == 1 ? b : c);
}

// repack points with x,y,z at offsets 0,4,8 (+ intensity at 16 for a 32-byte PCL stride, at 12 for
// 16-byte packing) into packed float4
void repack(const float* src, size_t n, size_t stride, float4* out) {
    if (stride == 16) {
        if (n) std::memcpy(out, src, sizeof(float4) * n);
        return;
    }
    const char* b = reinterpret_cast<const char*>(src);
    for (size_t i = 0; i < n; ++i) {
        const float* p = reinterpret_cast<const float*>(b + i * stride);
        float inten = 0.f;
        if (stride >= 20) inten = p[4];
        else if (stride >= 16) inten = p[3];
        out[i] = make_float4(p[0], p[1], p[2], inten);
    }
}

bool valid_stride(size_t s) { return s == 16 || s == 32 || s >= 12; }

// pf_host_alloc blocks (pinned, mapped, portable): host base -> (bytes, device-side address). Host-input
// entry points DMA straight from such a block instead of repacking the caller's memory first.
struct PinnedBlock {
    size_t bytes;
    char* dev;
};
std::mutex g_pin_mu;
std::map<uintptr_t, PinnedBlock> g_pinned;

// the device-side address of [p, p + bytes) when it lies inside one pf_host_alloc block, else nullptr
void* pinned_dev(const void* p, size_t bytes) {
    if (!p) return nullptr;
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pinned.upper_bound((uintptr_t)p);
    if (it == g_pinned.begin()) return nullptr;
    --it;
    const uintptr_t a = (uintptr_t)p;
    if (a + bytes > it->first + it->second.bytes) return nullptr;
    return it->second.dev + (a - it->first);
}

// read_pose's one gather: counters, sticky error words, the latest pose (identity before the first
// frame) and the estimator state into mapped pinned host memory
__global__ void k_readback(const int* __restrict__ cnt, const int* __restrict__ errw, const double* __restrict__ pose,
                           const DevState* __restrict__ st, HostRead* __restrict__ out) {
    const int t = threadIdx.x;
    if (t < C_COUNT) out->cnt[t] = cnt[t];
    if (t < E_COUNT) out->err[t] = errw[t];
    if (t < 7) out->pose[t] = pose ? pose[t] : (t == 3 ? 1.0 : 0.0);
    constexpr int nw = (int)(sizeof(DevState) / 4);
    for (int i = t; i < nw; i += blockDim.x) reinterpret_cast<int*>(&out->st)[i] = reinterpret_cast<const int*>(st)[i];
}

// fe handle output: the counts and, when they fit `cap`, the edge / surf points into the caller's
// (mapped) memory or the handle's mapped staging; one launch after featureExtraction, no count round trip
__global__ void k_fe_out(const int* __restrict__ cnt, const int* __restrict__ ferr, const float4* __restrict__ e,
                         const float4* __restrict__ sf, float4* __restrict__ oe, float4* __restrict__ os, int cap,
                         int* __restrict__ hcnt) {
    const int ne = cnt[1], ns = cnt[2];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        hcnt[0] = ne;
        hcnt[1] = ns;
        hcnt[2] = *ferr;
    }
    if (ne > cap || ns > cap) return;
    const int stride = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ne + ns; i += stride) {
        if (i < ne) oe[i] = e[i];
        else os[i - ne] = sf[i - ne];
    }
}

}  // namespace

struct pf_fe {
    int device = 0;
    hipStream_t stream = nullptr;
    FeGPU fe;
    float4* d_edge = nullptr;
    float4* d_surf = nullptr;
    int* d_cnt = nullptr;   // [0] n, [1] ne, [2] ns
    int* h_cnt = nullptr;   // mapped pinned: ne, ns, featureExtraction error word
    int* h_cnt_dev = nullptr;
    float4* h_in = nullptr;   // pinned staging of a repacked scan (max_points)
    float4* h_out = nullptr;  // mapped pinned staging of the outputs (2 x max_points)
    float4* h_out_dev = nullptr;
};

// per-stage device timing (pf_odom_set_stage_timing): a ring of event quadruples {A start, A end,
// B start, B end}; a quadruple is harvested (its elapsed times summed) before its ring slot is reused
struct StageTiming {
    static constexpr int kRing = 256;
    bool on = false;
    hipEvent_t ev[kRing][4] = {};
    bool pending[kRing] = {};
    long long next = 0;
    double sum_a = 0, sum_b = 0;
    size_t frames = 0;
};

struct pf_odom {
    OdomGPU o;
    StageTiming* timing = nullptr;
    bool counted = false;      // in g_live_handles
    bool front_counted = false;  // in g_front_handles (has run the BPF raw-scan front end)
};

static int timing_harvest(StageTiming& t, int j) {
    if (!t.pending[j]) return PF_OK;
    PF_HIP_TRY(hipEventSynchronize(t.ev[j][3]));
    float a = 0.f, b = 0.f;
    PF_HIP_TRY(hipEventElapsedTime(&a, t.ev[j][0], t.ev[j][1]));
    PF_HIP_TRY(hipEventElapsedTime(&b, t.ev[j][2], t.ev[j][3]));
    t.sum_a += 1e3 * a;
    t.sum_b += 1e3 * b;
    t.frames++;
    t.pending[j] = false;
    return PF_OK;
}
static void timing_free(pf_odom* h) {
    if (!h->timing) return;
    for (auto& q : h->timing->ev)
        for (hipEvent_t& e : q)
            if (e) (void)hipEventDestroy(e);
    delete h->timing;
    h->timing = nullptr;
}
// marks k = 0..3 (A start, A end, B start, B end) of the current frame
static int timing_mark(pf_odom* h, int k, hipStream_t s = nullptr) {
    StageTiming* t = h->timing;
    if (!t || !t->on) return PF_OK;
    const int j = (int)(t->next % StageTiming::kRing);
    if (k == 0) {
        if (int rc = timing_harvest(*t, j)) return rc;
    }
    PF_HIP_TRY(hipEventRecord(t->ev[j][k], s ? s : (k < 2 ? h->o.stream_a : h->o.stream)));
    if (k == 3) {
        t->pending[j] = true;
        t->next++;
    }
    return PF_OK;
}


extern "C" {

// ------------------------------------------------------------------------------------------------
int pf_fe_create(const pf_lidar_params* lidar, int device, size_t max_points, pf_fe** out) {
    if (!lidar || !out || max_points == 0) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(device));
    pf_fe* h = new (std::nothrow) pf_fe();
    if (!h) return PF_ENOMEM;
    h->device = device;
    int rc = fe_alloc(h->fe, *lidar, max_points);
    h->fe.tie_order = true;               // the reference's std::sort order by default (pf_fe_set_tie_order)
    const size_t ecap = (size_t)h->fe.rings * 6 * kEdgePerSector;
    if (rc == PF_OK && hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) rc = PF_EHIP;
    if (rc == PF_OK && hipMalloc(&h->d_edge, sizeof(float4) * ecap) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_surf, sizeof(float4) * max_points) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_cnt, sizeof(int) * 4) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipHostMalloc(&h->h_cnt, sizeof(int) * 4, hipHostMallocMapped) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipHostGetDevicePointer(reinterpret_cast<void**>(&h->h_cnt_dev), h->h_cnt, 0) != hipSuccess)
        rc = PF_EHIP;
    if (rc == PF_OK && hipHostMalloc(&h->h_in, sizeof(float4) * max_points) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipHostMalloc(&h->h_out, sizeof(float4) * 2 * max_points, hipHostMallocMapped) != hipSuccess)
        rc = PF_ENOMEM;
    if (rc == PF_OK && hipHostGetDevicePointer(reinterpret_cast<void**>(&h->h_out_dev), h->h_out, 0) != hipSuccess)
        rc = PF_EHIP;
    if (rc != PF_OK) {
        pf_fe_destroy(h);
        return rc;
    }
    *out = h;
    return PF_OK;
}

int pf_fe_destroy(pf_fe* h) {
    if (!h) return PF_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    fe_free(h->fe);
    (void)hipFree(h->d_edge);
    (void)hipFree(h->d_surf);
    (void)hipFree(h->d_cnt);
    if (h->h_cnt) (void)hipHostFree(h->h_cnt);
    if (h->h_in) (void)hipHostFree(h->h_in);
    if (h->h_out) (void)hipHostFree(h->h_out);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return PF_OK;
}

// One synchronisation per call: the scan goes up by DMA (straight from a pf_host_alloc block with a
// 16-byte stride, else repacked into pinned staging first), featureExtraction runs, and k_fe_out writes
// the counts and the clouds into mapped host memory (the caller's own pf_host_alloc outputs, or the
// handle's staging, copied out after the synchronisation).
int pf_fe_extract(pf_fe* h, const float* xyzi, size_t n, size_t stride_bytes, float* edge_out, size_t* n_edge,
                  float* surf_out, size_t* n_surf, size_t cap) {
    if (!h || (!xyzi && n) || !n_edge || !n_surf || !valid_stride(stride_bytes)) return PF_EINVAL;
    if (n > h->fe.cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(h->device));
    if (n) {
        const void* src = stride_bytes == 16 && pinned_dev(xyzi, sizeof(float4) * n) ? (const void*)xyzi : nullptr;
        if (!src) {
            repack(xyzi, n, stride_bytes, h->h_in);
            src = h->h_in;
        }
        PF_HIP_TRY(hipMemcpyAsync(h->fe.d_in_stage, src, sizeof(float4) * n, hipMemcpyHostToDevice, h->stream));
    }
    hipLaunchKernelGGL(k_set_int, dim3(1), dim3(64), 0, h->stream, h->d_cnt, (int)n);
    fe_enqueue(h->fe, h->fe.d_in_stage, h->d_cnt, h->d_edge, h->d_cnt + 1, h->d_surf, h->d_cnt + 2, h->stream);
    const size_t ocap = cap < (size_t)INT_MAX ? cap : (size_t)INT_MAX;
    float4* de = edge_out ? static_cast<float4*>(pinned_dev(edge_out, sizeof(float4) * ocap)) : nullptr;
    float4* ds = surf_out ? static_cast<float4*>(pinned_dev(surf_out, sizeof(float4) * ocap)) : nullptr;
    hipLaunchKernelGGL(k_fe_out, dim3(256), dim3(256), 0, h->stream, h->d_cnt, h->fe.err, h->d_edge, h->d_surf,
                       de ? de : h->h_out_dev, ds ? ds : h->h_out_dev + h->fe.cap, (int)ocap, h->h_cnt_dev);
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    PF_HIP_TRY(hipGetLastError());
    if (h->h_cnt[2]) {
        PF_HIP_TRY(hipMemsetAsync(h->fe.err, 0, sizeof(int), h->stream));
        return PF_EUNSUPPORTED;
    }
    const size_t ne = (size_t)h->h_cnt[0], ns = (size_t)h->h_cnt[1];
    *n_edge = ne;
    *n_surf = ns;
    if (ne > cap || ns > cap) return PF_ECAPACITY;
    if (edge_out && !de && ne) std::memcpy(edge_out, h->h_out, sizeof(float4) * ne);
    if (surf_out && !ds && ns) std::memcpy(surf_out, h->h_out + h->fe.cap, sizeof(float4) * ns);
    return PF_OK;
}

int pf_fe_set_ring_model(pf_fe* h, double top_deg, double bottom_deg) {
    if (!h) return PF_EINVAL;
    return fe_set_ring_model(h->fe, top_deg, bottom_deg);
}

int pf_fe_set_tie_order(pf_fe* h, int enable) {
    if (!h) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->device));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    h->fe.tie_order = enable != 0;
    return PF_OK;
}

// ------------------------------------------------------------------------------------------------
// live handles of the process (PF_GRAPH_AUTO: stage B replays its graph when several handles share
// the host's launch path)
static std::atomic<int> g_live_handles{0};
// handles of this process with a BPF raw-scan front end: the auto lane mode gives two front-end lanes
// only while one such handle exists (idle ES handles in the same process do not count)
static std::atomic<int> g_front_handles{0};

static int create(const pf_lidar_params* lidar, const pf_odom_params* params, int device, size_t max_points,
                  size_t map_capacity, int nc, pf_odom** out) {
    if (!lidar || !params || !out) return PF_EINVAL;
    const int wt = params->weight_type;
    if (!(wt == 0 || wt == 1 || wt == 2 || wt == 12)) return PF_EINVAL;   // reference: ROS_ERROR + UB
    if (!(params->map_res > 0)) return PF_EINVAL;
    if (max_points == 0) max_points = 300000;
    if (map_capacity == 0) map_capacity = (size_t)1 << 22;
    PF_HIP_TRY(hipSetDevice(device));
    pf_odom* h = new (std::nothrow) pf_odom();
    if (!h) return PF_ENOMEM;
    int rc = odom_create(h->o, *lidar, *params, device, max_points, map_capacity, nc);
    // the reference's results by default: VoxelGrid / rgbds / the sector sort in std::sort's order of
    // equal keys (pf_odom_set_tie_order(h, 0) selects the stable sorts). A sort capacity past the tie
    // sort's per-level big-segment list (tie_alloc: PF_EINVAL from about 32M elements, i.e. map_capacity
    // of about 16M for ES / 10.5M for BPF) keeps the handle in the stable order rather than failing the
    // create, as before round 5; pf_odom_set_tie_order(h, 1) then returns PF_EINVAL for it
    if (rc == PF_OK) {
        rc = pf_odom_set_tie_order(h, 1);
        if (rc == PF_EINVAL) rc = PF_OK;
    }
    if (rc != PF_OK) {
        pf_odom_destroy(h);
        return rc;
    }
    h->counted = true;
    g_live_handles.fetch_add(1);
    *out = h;
    return PF_OK;
}

int pf_odom_create(const pf_lidar_params* lidar, const pf_odom_params* params, int device, size_t max_points,
                   size_t map_capacity, pf_odom** out) {
    return create(lidar, params, device, max_points, map_capacity, 2, out);
}

int pf_bpf_create(const pf_lidar_params* lidar, const pf_odom_params* params, int device, size_t max_points,
                  size_t map_capacity, pf_odom** out) {
    return create(lidar, params, device, max_points, map_capacity, 3, out);
}

int pf_odom_classes(pf_odom* h) { return h ? h->o.cls.nc : PF_EINVAL; }

static void host_prof_report();

int pf_odom_destroy(pf_odom* h) {
    if (!h) return PF_OK;
    (void)hipSetDevice(h->o.device);
    (void)odom_sync_a(h->o);
    (void)hipStreamSynchronize(h->o.stream);
    timing_free(h);
    host_prof_report();
    odom_destroy(h->o);
    if (h->counted) g_live_handles.fetch_sub(1);
    if (h->front_counted) g_front_handles.fetch_sub(1);
    delete h;
    return PF_OK;
}

int pf_odom_reset(pf_odom* h) {
    if (!h) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    return odom_reset(h->o);
}

// Frame k uses pipeline slot k % kSlots. Stage A (featureExtraction / VoxelGrid or host staging) of
// slot p first waits until stage B has finished frame k - kSlots (the previous user of the slot);
// stage B of frame k waits for stage A of frame k. Consecutive frames thus overlap A(k) with B(k - 1),
// and stage A may run up to kSlots - 1 frames ahead.
static int stage_a_begin(pf_odom* h, int p) {
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipStreamWaitEvent(o.stream_a, o.ev_b[p], 0));
    return PF_OK;
}
static int stage_a_end_b_begin(pf_odom* h, int p) {
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipEventRecord(o.ev_a[p], o.stream_a));
    PF_HIP_TRY(hipStreamWaitEvent(o.stream, o.ev_a[p], 0));
    return PF_OK;
}
static int stage_b_end(pf_odom* h, int p) {
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipEventRecord(o.ev_b[p], o.stream));
    o.frames++;
    return PF_OK;
}

// Host-input staging (HostStage), allocated by the first host-input call of a handle
static int host_stage(OdomGPU& o) {
    if (o.hs) return PF_OK;
    HostStage* hs = new (std::nothrow) HostStage();
    if (!hs) return PF_ENOMEM;
    o.hs = hs;              // freed by odom_destroy, also after a partial allocation
    const size_t pts = (size_t)kMaxC * o.in_cap;
    if (hipStreamCreateWithFlags(&hs->stream, hipStreamNonBlocking) != hipSuccess) return PF_EHIP;
    for (int p = 0; p < kSlots; ++p) {
        if (hipHostMalloc(&hs->h[p], sizeof(float4) * pts) != hipSuccess) return PF_ENOMEM;
        if (hipMalloc(&hs->d[p], sizeof(float4) * pts) != hipSuccess) return PF_ENOMEM;
        if (hipEventCreateWithFlags(&hs->ev[p], hipEventDisableTiming) != hipSuccess) return PF_EHIP;
    }
    return PF_OK;
}

// Uploads nc host clouds for the frame in slot p into hs->d[p] (cloud c at offset c * in_cap) on the
// copy stream and makes stage A's stream wait for the copy. A cloud with a 16-byte stride inside a
// pf_host_alloc block goes up straight from the caller's memory; any other is repacked into the
// slot's pinned buffer first. The device slot is rewritten only after stage A of the slot's previous
// frame (ev_a[p]) and the pinned slot only after its previous copy (hs->ev[p]), so neither the host
// nor the streams wait for each other in steady state. *direct: some cloud was read from the caller's
// memory (the caller must wait for hs->ev[p] before its buffers may change).
static int host_upload(OdomGPU& o, int p, int nc, const float* const* cl, const size_t* n, const size_t* stride,
                       bool* direct, float4* const* dst_dev = nullptr) {
    if (int rc = host_stage(o)) return rc;
    HostStage& hs = *o.hs;
    *direct = false;
    bool repacked = false;
    for (int c = 0; c < nc; ++c) {
        if ((!cl[c] && n[c]) || !valid_stride(stride[c])) return PF_EINVAL;
        if (n[c] > o.in_cap) return PF_ECAPACITY;
    }
    PF_HIP_TRY(hipStreamWaitEvent(hs.stream, o.ev_a[p], 0));
    // straight into the slot's stage inputs: stage B of the slot's previous frame may still read them
    // (k_init_map after an asynchronous first frame)
    if (dst_dev) PF_HIP_TRY(hipStreamWaitEvent(hs.stream, o.ev_b[p], 0));
    for (int c = 0; c < nc; ++c) {
        if (!n[c]) continue;
        const void* src = stride[c] == 16 && pinned_dev(cl[c], sizeof(float4) * n[c]) ? (const void*)cl[c] : nullptr;
        if (src) {
            *direct = true;
        } else {
            if (!repacked) PF_HIP_TRY(hipEventSynchronize(hs.ev[p]));   // the pinned slot's last copy is done
            repacked = true;
            float4* dst = hs.h[p] + (size_t)c * o.in_cap;
            repack(cl[c], n[c], stride[c], dst);
            src = dst;
        }
        PF_HIP_TRY(hipMemcpyAsync(dst_dev ? dst_dev[c] : hs.d[p] + (size_t)c * o.in_cap, src, sizeof(float4) * n[c],
                                  hipMemcpyHostToDevice, hs.stream));
    }
    PF_HIP_TRY(hipEventRecord(hs.ev[p], hs.stream));
    PF_HIP_TRY(hipStreamWaitEvent(o.stream_a, hs.ev[p], 0));
    return PF_OK;
}

// the caller's class clouds (host memory) straight into slot p's inputs (the copy stream waits for the
// slot's previous stage A and stage B, stage A's stream for the copies). The callers (init_map_n /
// update_n) return after a readback of stage B, which waits for stage A and so for these copies: the
// caller's buffers are free on return without a wait here. On their early-return paths the copies may
// still be reading the caller's memory (*direct): they wait for them first (inputs_done).
static int stage_inputs(pf_odom* h, int p, const float* const* cl, const size_t* n, const size_t* stride,
                        bool* direct) {
    OdomGPU& o = h->o;
    const int nc = o.cls.nc;
    StageBuf& sb = o.sb[p];
    *direct = false;
    if (int rc = host_upload(o, p, nc, cl, n, stride, direct, sb.in)) return rc;
    int cnt[kMaxC] = {0, 0, 0};
    for (int c = 0; c < nc; ++c) cnt[c] = (int)n[c];
    hipLaunchKernelGGL(k_set_counts, dim3(1), dim3(64), 0, o.stream_a, sb.cnt + C_IN, cnt[0], cnt[1], cnt[2], nc);
    return PF_OK;
}

// The handle's sticky error words (ErrWord, pf_odom.h) as read into e[0 .. E_COUNT): any word set since
// the last report is reported once and cleared. A bounded device wait that gave up (LM chunks, sort
// look-back) is PF_EHIP; a dropped sector, an overfull map grid or a front-end grid limit is PF_ECAPACITY.
// `peek` reads without reporting (get_stats).
static int sticky_report(OdomGPU& o, const int* e, bool peek) {
    int bits = 0;
    for (int k = 0; k < E_COUNT; ++k)
        if (e[k]) bits |= 1 << k;
    o.err_seen |= bits;
    if (!bits || peek) return PF_OK;
    for (int k = 0; k < E_COUNT; ++k) o.err_last[k] = e[k];
    PF_HIP_TRY(hipMemsetAsync(o.errw, 0, sizeof(int) * E_COUNT, o.stream));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    const int hip_bits = (1 << E_LM) | (1 << E_SORT_A) | (1 << E_SORT_B);
    return (bits & hip_bits) ? PF_EHIP : PF_ECAPACITY;
}

// the sticky words read on stage B's stream after the work enqueued so far
static int sticky_status(OdomGPU& o, bool peek = false) {
    int* e = o.h_cnt + C_COUNT;
    PF_HIP_TRY(hipMemcpyAsync(e, o.errw, sizeof(int) * E_COUNT, hipMemcpyDeviceToHost, o.stream));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    return sticky_report(o, e, peek);
}

// After the work enqueued so far: counters, error words, the latest pose and the estimator state in
// one gather (k_readback) and one synchronisation; reports the sticky words. The state read stays
// cached for pf_odom_get_state until the next frame / update / set_state.
static void drop_graphs_b(OdomGPU& o);
static int readback(pf_odom* h) {
    OdomGPU& o = h->o;
    const double* pose = o.frames > 0 ? o.poses + 7 * ((size_t)(o.frames - 1) % o.pose_cap) : nullptr;
    hipLaunchKernelGGL(k_readback, dim3(1), dim3(64), 0, o.stream, o.cnt, o.errw, pose, o.st, o.h_rd_dev);
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    PF_HIP_TRY(hipGetLastError());
    o.rd_frames = o.frames;
    // a map grown past the tie sort's big-level threshold since the last hint (pf_odom_set_map raises it
    // at once): the next rgbds sorts start in big levels, so the captured stage B is re-captured
    if (o.tie_b) {
        size_t mx = 0;
        for (int c = 0; c < o.cls.nc; ++c) mx = std::max(mx, (size_t)o.h_rd->cnt[C_M + c] + (size_t)o.h_rd->cnt[C_DS + c]);
        if (mx > o.tie_hint && tie_levels_for(*o.tie_b, mx + 65536) != tie_levels_for(*o.tie_b, o.tie_hint)) {
            o.tie_hint = mx + 65536;
            drop_graphs_b(o);
        }
    }
    return sticky_report(o, o.h_rd->err, false);
}

static int read_pose(pf_odom* h, double pose[7]) {
    const int rc = readback(h);
    std::memcpy(pose, h->o.h_rd->pose, sizeof(double) * 7);
    return rc;
}

// the update / init_map status from the counters of the last readback: the reference's messages
static int frame_status(pf_odom* h) {
    const int* c = h->o.h_rd->cnt;
    if (c[C_ERR]) return PF_EHIP;                        // a bounded device-side wait gave up
    if (!c[C_GATE]) return PF_W_MAP_TOO_SMALL;
    for (int k = 0; k < h->o.cls.nc; ++k)              // :428-431 / :574-577, BPF :875-878, :1188-1191
        if (c[C_KEPT + k] < 20) return PF_W_FEW_CORRESPONDENCES;
    return PF_OK;
}

// an early return after stage_inputs: the copies from the caller's memory complete first
static int inputs_done(pf_odom* h, int p, bool direct, int rc) {
    if (direct && h->o.hs) (void)hipEventSynchronize(h->o.hs->ev[p]);
    return rc;
}

static int init_map_n(pf_odom* h, const float* const* cl, const size_t* n, const size_t* stride) {
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    const int p = o.frames % kSlots;
    bool direct = false;
    int rc = stage_a_begin(h, p);
    if (!rc) rc = stage_inputs(h, p, cl, n, stride, &direct);
    if (!rc) rc = stage_a_end_b_begin(h, p);
    if (rc) return inputs_done(h, p, direct, rc);
    odom_enqueue_init(o, p, o.stream);
    odom_enqueue_export(o, o.stream, false);
    rc = stage_b_end(h, p);
    if (rc) return inputs_done(h, p, direct, rc);
    return inputs_done(h, p, direct, readback(h));
}

// updatePointsToMap is synchronous in the reference (the node reads `odom` right after it): one
// readback per call reports the pose, the status and the sticky words
static int update_n(pf_odom* h, const float* const* cl, const size_t* n, const size_t* stride, double pose_out[7]) {
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    const int p = o.frames % kSlots;
    bool direct = false;
    int rc = stage_a_begin(h, p);
    if (!rc) rc = stage_inputs(h, p, cl, n, stride, &direct);
    if (rc) return inputs_done(h, p, direct, rc);
    stage_enqueue_vg(o, p, o.stream_a);
    rc = stage_a_end_b_begin(h, p);
    if (rc) return inputs_done(h, p, direct, rc);
    odom_enqueue_update(o, p, o.stream);
    odom_enqueue_export(o, o.stream, true);
    odom_update_done(o);
    rc = stage_b_end(h, p);
    if (rc) return inputs_done(h, p, direct, rc);
    rc = inputs_done(h, p, direct, readback(h));
    if (pose_out) std::memcpy(pose_out, o.h_rd->pose, sizeof(double) * 7);
    if (rc) return rc;
    return frame_status(h);
}

int pf_odom_init_map(pf_odom* h, const float* edge, size_t ne, size_t edge_stride, const float* surf, size_t ns,
                     size_t surf_stride) {
    if (!h || h->o.cls.nc != 2) return PF_EINVAL;
    const float* cl[2] = {edge, surf};
    const size_t n[2] = {ne, ns}, st[2] = {edge_stride, surf_stride};
    return init_map_n(h, cl, n, st);
}

int pf_odom_update(pf_odom* h, const float* edge, size_t ne, size_t edge_stride, const float* surf, size_t ns,
                   size_t surf_stride, double pose_out[7]) {
    if (!h || h->o.cls.nc != 2) return PF_EINVAL;
    const float* cl[2] = {edge, surf};
    const size_t n[2] = {ne, ns}, st[2] = {edge_stride, surf_stride};
    return update_n(h, cl, n, st, pose_out);
}

int pf_bpf_init_map(pf_odom* h, const float* beam, size_t nb, size_t beam_stride, const float* pillar, size_t np,
                    size_t pillar_stride, const float* facade, size_t nf, size_t facade_stride) {
    if (!h || h->o.cls.nc != 3) return PF_EINVAL;
    const float* cl[3] = {beam, pillar, facade};
    const size_t n[3] = {nb, np, nf}, st[3] = {beam_stride, pillar_stride, facade_stride};
    return init_map_n(h, cl, n, st);
}

int pf_bpf_update(pf_odom* h, const float* beam, size_t nb, size_t beam_stride, const float* pillar, size_t np,
                  size_t pillar_stride, const float* facade, size_t nf, size_t facade_stride, double pose_out[7]) {
    if (!h || h->o.cls.nc != 3) return PF_EINVAL;
    const float* cl[3] = {beam, pillar, facade};
    const size_t n[3] = {nb, np, nf}, st[3] = {beam_stride, pillar_stride, facade_stride};
    return update_n(h, cl, n, st, pose_out);
}

int pf_odom_get_pose(pf_odom* h, double pose[7]) {
    if (!h || !pose) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    return read_pose(h, pose);
}

int pf_odom_get_map(pf_odom* h, int which, float* xyz, uint8_t* rg, size_t cap, size_t* n) {
    if (!h || !n || which < 0 || which >= h->o.cls.nc) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(hipMemcpyAsync(o.h_cnt, o.cnt, sizeof(int) * C_COUNT, hipMemcpyDeviceToHost, o.stream));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    const size_t m = (size_t)o.h_cnt[C_M + which];
    *n = m;
    if (!xyz && !rg) return PF_OK;
    if (m > cap) return PF_ECAPACITY;
    std::vector<float4> tmp(m);
    if (m) {
        PF_HIP_TRY(hipMemcpyAsync(tmp.data(), map_cur(o)[which], sizeof(float4) * m, hipMemcpyDeviceToHost, o.stream));
        PF_HIP_TRY(hipStreamSynchronize(o.stream));
    }
    for (size_t i = 0; i < m; ++i) {
        if (xyz) { xyz[3 * i] = tmp[i].x; xyz[3 * i + 1] = tmp[i].y; xyz[3 * i + 2] = tmp[i].z; }
        if (rg) {
            uint32_t w;
            std::memcpy(&w, &tmp[i].w, 4);
            rg[2 * i] = (uint8_t)(w & 255u);
            rg[2 * i + 1] = (uint8_t)((w >> 8) & 255u);
        }
    }
    return PF_OK;
}

int pf_odom_set_map(pf_odom* h, int which, const float* xyz, const uint8_t* rg, size_t n) {
    if (!h || which < 0 || which >= h->o.cls.nc || (!xyz && n)) return PF_EINVAL;
    OdomGPU& o = h->o;
    if (n > o.map_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(o.device));
    std::vector<float4> tmp(n);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t w = rg ? pack_rg(rg[2 * i], rg[2 * i + 1]) : 0u;
        float wf;
        std::memcpy(&wf, &w, 4);
        tmp[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], wf);
    }
    if (n) PF_HIP_TRY(hipMemcpyAsync(map_cur(o)[which], tmp.data(), sizeof(float4) * n, hipMemcpyHostToDevice, o.stream));
    hipLaunchKernelGGL(k_set_int, dim3(1), dim3(64), 0, o.stream, o.cnt + C_M + which, (int)n);
    odom_dep_dirty(o, o.stream);                        // any points, several per voxel maybe
    o.dims_fresh = false;                               // the next update's grid takes its bounds pass
    if (n + 65536 > o.tie_hint) o.tie_hint = n + 65536;  // the tie-order rgbds sort starts in big levels above kTieMed
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    return PF_OK;
}

int pf_odom_get_stats(pf_odom* h, pf_odom_stats* s) {
    if (!h || !s) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(hipMemcpyAsync(o.h_cnt, o.cnt, sizeof(int) * C_COUNT, hipMemcpyDeviceToHost, o.stream));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    const int* c = o.h_cnt;
    std::memset(s, 0, sizeof(*s));
    for (int k = 0; k < o.cls.nc; ++k) {
        s->n_in[k] = c[C_IN + k];
        s->n_ds[k] = c[C_DS + k];
        s->n_map[k] = c[C_M + k];
        s->n_res[k] = c[C_KEPT + k];
        s->n_valid[k] = c[C_VALID + k];
    }
    s->n_edge_in = s->n_in[0];          // ES names: class 0 = edge (corner), class 1 = surf
    s->n_surf_in = s->n_in[1];
    s->n_edge_ds = s->n_ds[0];
    s->n_surf_ds = s->n_ds[1];
    s->n_edge_map = s->n_map[0];
    s->n_surf_map = s->n_map[1];
    s->n_edge_res = s->n_res[0];
    s->n_surf_res = s->n_res[1];
    s->n_edge_valid = s->n_valid[0];
    s->n_surf_valid = s->n_valid[1];
    s->outer_iterations = c[C_OUTER];
    s->lm_iterations = c[C_LM_ITERS];
    s->map_too_small = c[C_GATE] ? 0 : 1;
    if (int rc = sticky_status(o, true)) return rc;
    s->errors = o.err_seen;
    return PF_OK;
}

// ------------------------------------------------------------------------------------------------
// whole frame on the device, as two pipelined stages. In steady state (optimization_count == 2)
// each stage replays a hipGraph captured once per slot; the scan is first copied into the handle's
// fixed staging buffer and its size written to the slot's counters (both outside the graph).
// BPF raw-scan mode, stage A head: the front end (ground_seg + featureExtract) of the staged scan
// writes slot p's beam / pillar / facade clouds and their device-resident sizes
static void stage_enqueue_front(OdomGPU& o, int p, hipStream_t s) {
    float4* out[3] = {o.sb[p].in[0], o.sb[p].in[1], o.sb[p].in[2]};
    int* cnt[3] = {o.sb[p].cnt + C_IN, o.sb[p].cnt + C_IN + 1, o.sb[p].cnt + C_IN + 2};
    cls_enqueue(*o.front, o.stage, o.sb[p].cnt + C_NIN, out, cnt, false, s);
}

// front-end lane `lane` of the frame in slot p: the staged scan of that lane through its instance
static void stage_enqueue_front_lane(OdomGPU& o, int p, int lane, hipStream_t s) {
    float4* out[3] = {o.sb[p].in[0], o.sb[p].in[1], o.sb[p].in[2]};
    int* cnt[3] = {o.sb[p].cnt + C_IN, o.sb[p].cnt + C_IN + 1, o.sb[p].cnt + C_IN + 2};
    cls_enqueue(lane ? *o.front2 : *o.front, lane ? o.stage2 : o.stage, o.sb[p].cnt + C_NIN, out, cnt, false, s);
}

static void drop_graphs_f(OdomGPU& o) {
    for (hipGraphExec_t& g : o.graph_f)
        if (g) {
            (void)hipGraphExecDestroy(g);
            g = nullptr;
        }
}

// The second front-end lane of a BPF raw-scan handle (OdomGPU::front_lanes): both lanes' streams
// (stage A's CU mask), the slot events, and lane 1's front end (lane 0's parameters and DCVC) and
// scan staging. Called by the first raw-scan frame with two lanes.
static int front_lanes_ready(OdomGPU& o) {
    if (o.front2) return PF_OK;
    for (int l = 0; l < 2; ++l)
        if (!o.stream_f[l])
            if (int rc = odom_masked_stream(o.device, o.cu_reserve, &o.stream_f[l])) return rc;
    for (int p = 0; p < kSlots; ++p)
        if (!o.ev_f[p]) PF_HIP_TRY(hipEventCreateWithFlags(&o.ev_f[p], hipEventDisableTiming));
    if (!o.stage2) PF_HIP_TRY(hipMalloc(&o.stage2, sizeof(float4) * kMaxC * o.in_cap));
    ClsGPU* f = new (std::nothrow) ClsGPU();
    if (!f) return PF_ENOMEM;
    int rc = cls_alloc(*f, o.in_cap);
    if (!rc) {
        f->prm = o.front->prm;
        f->sticky = o.errw + E_FRONT;
        alias_err(f->grid.err, o.errw + E_FRONT_GRID);
        if (o.front->dcvc) {
            rc = cls_set_dcvc(*f, &o.front->dcvc->prm);
            if (!rc) rc = dcvc_mark_called(*f->dcvc, o.stream_f[1]);
        }
    }
    if (rc) {
        if (f->grid.err == o.errw + E_FRONT_GRID) f->grid.err = nullptr;
        cls_free(*f);
        delete f;
        return rc;
    }
    o.front2 = f;
    return PF_OK;
}

static void drop_graphs_b(OdomGPU& o) {
    for (hipGraphExec_t& g : o.graph_b)
        if (g) {
            (void)hipGraphExecDestroy(g);
            g = nullptr;
        }
}

static int capture(hipStream_t s, hipGraphExec_t* out, OdomGPU& o, int p, bool stage_a, bool scan = false) {
    hipGraph_t g;
    PF_HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    if (stage_a) {
        if (o.cls.nc == 2) stage_enqueue_fe(o, p, o.stage, s);
        else if (scan) stage_enqueue_front(o, p, s);
        stage_enqueue_vg(o, p, s);
    } else {
        odom_enqueue_update(o, p, s);
        odom_enqueue_export(o, s, true);
    }
    PF_HIP_TRY(hipStreamEndCapture(s, &g));
    PF_HIP_TRY(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    return PF_OK;
}

static int capture_front(hipStream_t s, hipGraphExec_t* out, OdomGPU& o, int p, int lane) {
    hipGraph_t g;
    PF_HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    stage_enqueue_front_lane(o, p, lane, s);
    PF_HIP_TRY(hipStreamEndCapture(s, &g));
    PF_HIP_TRY(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    return PF_OK;
}

// development: PF_HOST_PROFILE=1 prints the mean host time of every HIP call site of enqueue_frame
// when the handle is destroyed
struct HostProf {
    static constexpr int kSites = 8;
    double us[kSites] = {};
    long long n[kSites] = {};
    std::vector<float> samp[kSites];
    bool on = std::getenv("PF_HOST_PROFILE") != nullptr;
};
static HostProf g_hprof;
#define PF_HT(site, expr)                                                                        \
    do {                                                                                         \
        if (!g_hprof.on) { expr; break; }                                                        \
        const auto t0_ = std::chrono::steady_clock::now();                                       \
        expr;                                                                                    \
        const double dt_ = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0_).count(); \
        g_hprof.us[site] += dt_;                                                                 \
        g_hprof.n[site]++;                                                                       \
        g_hprof.samp[site].push_back((float)dt_);                                                \
    } while (0)
static void host_prof_report() {
    if (!g_hprof.on) return;
    static const char* names[HostProf::kSites] = {"wait ev_b", "scan D2D copy", "k_set_int", "graph A",
                                                 "record ev_a + wait", "graph B", "record ev_b", "whole call"};
    for (int k = 0; k < HostProf::kSites; ++k)
        if (g_hprof.n[k]) {
            std::vector<float>& v = g_hprof.samp[k];
            double first = 0;
            const size_t nf = v.size() < 100 ? v.size() : 100;
            for (size_t i = 0; i < nf; ++i) first += v[i];
            std::sort(v.begin(), v.end());
            auto q = [&](double f) { return v[(size_t)(f * (v.size() - 1))]; };
            std::fprintf(stderr,
                         "pf host profile: %-20s mean %8.2f us x %lld  p10 %.1f p50 %.1f p90 %.1f max %.1f  first100 "
                         "mean %.1f\n",
                         names[k], g_hprof.us[k] / g_hprof.n[k], g_hprof.n[k], q(0.1), q(0.5), q(0.9), q(1.0),
                         first / (nf ? nf : 1));
            v.clear();
        }
    g_hprof = HostProf{};
}

// one frame through both stages. ES: the raw scan d_in[0 .. n) is copied to the staging buffer and
// stage A runs featureExtraction + VoxelGrid. BPF: the class clouds cl[c][0 .. ncl[c]) are copied
// into the slot's inputs and stage A runs VoxelGrid; BPF raw-scan mode (cl null): the scan is staged
// as for ES and stage A runs the front end (pf_cls.h) then VoxelGrid. The copies and counts stay
// outside the graphs.
static int enqueue_frame(pf_odom* h, const float4* d_in, size_t n, const float4* const* cl, const size_t* ncl) {
    OdomGPU& o = h->o;
    const int nc = o.cls.nc;
    const bool scan = nc == 3 && !cl;
    const int p = o.frames % kSlots;
    // steady state: each stage replays its graph when its bit of the graph mode is set (graph B of the
    // merge path starts from the grid dims of the previous update: a frame after a host map write runs
    // eagerly)
    const bool steady = o.inited && o.opt_count_host <= 2;
    const int gm = o.graph_mode != PF_GRAPH_AUTO
                       ? o.graph_mode
                       : PF_GRAPH_STAGE_A | (g_live_handles.load(std::memory_order_relaxed) > 1 ? PF_GRAPH_STAGE_B : 0);
    const bool steady_a = steady && (gm & PF_GRAPH_STAGE_A);
    const bool steady_b = steady && (gm & PF_GRAPH_STAGE_B) && (o.dims_fresh || !odom_merge_mode(o));
    if (scan && n > o.in_cap) return PF_ECAPACITY;
    int rc = 0;
    const bool lanes = scan && (o.front_lanes == 2 ||
                                (o.front_lanes == 0 && g_front_handles.load(std::memory_order_relaxed) <= 1));
    if (lanes && (rc = front_lanes_ready(o))) return rc;
    if (scan && o.lanes_used != (lanes ? 2 : 1)) {
        // a change of lane mode: the instances the other mode used may still be busy (host wait, once)
        if (o.lanes_used) PF_HIP_TRY(odom_sync_a(o));
        o.lanes_used = lanes ? 2 : 1;
    }
    PF_HT(0, rc = stage_a_begin(h, p));
    if (rc) return rc;
    if (scan && o.dcvc_first && o.front->dcvc) {
        // the first curvedfilter frame since DCVC was enabled / reset: the instance of the lane that runs
        // it starts as never called (the reference's 5 m ring start, .hpp:105-106), every other instance
        // as called before, whichever lane the frame count gives: the reference has one curvedVoxel.
        // Each word is written on the stream of the lane that reads it, ahead of that lane's next frame.
        const int lane = lanes ? (o.frames & 1) : 0;
        ClsGPU* inst[2] = {o.front, o.front2};
        for (int q = 0; q < 2; ++q) {
            if (!inst[q] || !inst[q]->dcvc) continue;
            hipStream_t qs = lanes ? o.stream_f[q] : o.stream_a;
            if ((rc = q == lane ? dcvc_reset(*inst[q]->dcvc, qs) : dcvc_mark_called(*inst[q]->dcvc, qs))) return rc;
        }
        o.dcvc_first = false;
    }
    if (lanes) {
        // the front end on lane (frame & 1) once slot p is free, then VoxelGrid on stream_a in frame
        // order after it: two consecutive frames' front ends run at once
        const int lane = o.frames & 1;
        hipStream_t fs = o.stream_f[lane];
        PF_HIP_TRY(hipStreamWaitEvent(fs, o.ev_b[p], 0));
        if ((rc = timing_mark(h, 0, fs))) return rc;
        if (n) PF_HIP_TRY(hipMemcpyAsync(lane ? o.stage2 : o.stage, d_in, sizeof(float4) * n, hipMemcpyDeviceToDevice, fs));
        hipLaunchKernelGGL(k_set_int, dim3(1), dim3(64), 0, fs, o.sb[p].cnt + C_NIN, (int)n);
        if (steady_a) {
            hipGraphExec_t& gf = o.graph_f[p + kSlots * lane];
            if (!gf && (rc = capture_front(fs, &gf, o, p, lane))) return rc;
            PF_HIP_TRY(hipGraphLaunch(gf, fs));
        } else {
            stage_enqueue_front_lane(o, p, lane, fs);
        }
        PF_HIP_TRY(hipEventRecord(o.ev_f[p], fs));
        PF_HIP_TRY(hipStreamWaitEvent(o.stream_a, o.ev_f[p], 0));
        if (steady_a) {
            hipGraphExec_t& ga = o.graph_a[p];                 // nc == 3 without scan: VoxelGrid only
            if (!ga && (rc = capture(o.stream_a, &ga, o, p, true, false))) return rc;
            PF_HIP_TRY(hipGraphLaunch(ga, o.stream_a));
        } else if (o.inited) {
            stage_enqueue_vg(o, p, o.stream_a);
        }
    }
    if (!lanes && (rc = timing_mark(h, 0))) return rc;
    if (lanes) {
    } else if (nc == 2 || scan) {
        if (n > o.in_cap) return PF_ECAPACITY;
        if (n) PF_HT(1, PF_HIP_TRY(hipMemcpyAsync(o.stage, d_in, sizeof(float4) * n, hipMemcpyDeviceToDevice, o.stream_a)));
        PF_HT(2, hipLaunchKernelGGL(k_set_int, dim3(1), dim3(64), 0, o.stream_a, o.sb[p].cnt + C_NIN, (int)n));
    } else {
        for (int c = 0; c < nc; ++c) {
            if (ncl[c] > o.in_cap) return PF_ECAPACITY;
            if (ncl[c]) PF_HIP_TRY(hipMemcpyAsync(o.sb[p].in[c], cl[c], sizeof(float4) * ncl[c], hipMemcpyDeviceToDevice,
                                                  o.stream_a));
            hipLaunchKernelGGL(k_set_int, dim3(1), dim3(64), 0, o.stream_a, o.sb[p].cnt + C_IN + c, (int)ncl[c]);
        }
    }
    if (lanes) {
    } else if (steady_a) {
        hipGraphExec_t& ga = scan ? o.graph_as[p] : o.graph_a[p];
        if (!ga) {
            rc = capture(o.stream_a, &ga, o, p, true, scan);
            if (rc) return rc;
        }
        PF_HT(3, PF_HIP_TRY(hipGraphLaunch(ga, o.stream_a)));
    } else {
        if (nc == 2) stage_enqueue_fe(o, p, o.stage, o.stream_a);
        else if (scan) stage_enqueue_front(o, p, o.stream_a);
        if (o.inited) stage_enqueue_vg(o, p, o.stream_a);
    }
    rc = timing_mark(h, 1);
    if (!rc) PF_HT(4, rc = stage_a_end_b_begin(h, p));
    if (!rc) rc = timing_mark(h, 2);
    if (rc) return rc;
    if (steady_b) {
        hipGraphExec_t& gb = o.graph_b[p + kSlots * o.mpar];
        if (!gb) {
            rc = capture(o.stream, &gb, o, p, false);
            if (rc) return rc;
        }
        PF_HT(5, PF_HIP_TRY(hipGraphLaunch(gb, o.stream)));
        odom_update_done(o);
    } else if (!o.inited) {
        odom_enqueue_init(o, p, o.stream);
        odom_enqueue_export(o, o.stream, false);
    } else {
        odom_enqueue_update(o, p, o.stream);
        odom_enqueue_export(o, o.stream, true);
        odom_update_done(o);
    }
    rc = timing_mark(h, 3);
    if (rc) return rc;
    PF_HT(6, rc = stage_b_end(h, p));
    return rc;
}

int pf_odom_frame_device(pf_odom* h, const float* d_xyzi, size_t n, double pose_out[7]) {
    if (!h || (!d_xyzi && n) || h->o.cls.nc != 2) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    int rc = 0;
    PF_HT(7, rc = enqueue_frame(h, reinterpret_cast<const float4*>(d_xyzi), n, nullptr, nullptr));
    if (rc) return rc;
    if (pose_out) return read_pose(h, pose_out);
    return PF_OK;
}

// The scan goes up by DMA on the copy stream (host_upload) and stage A's stream waits for it: no host
// wait on the device. With pose_out NULL the call only enqueues (the frame pipeline of
// pf_odom_frame_device); from a pf_host_alloc block with a 16-byte stride the call returns once the
// DMA has read the caller's scan, otherwise once the scan is repacked into pinned staging.
int pf_odom_frame_host(pf_odom* h, const float* xyzi, size_t n, size_t stride_bytes, double pose_out[7]) {
    if (!h || (!xyzi && n) || !valid_stride(stride_bytes) || h->o.cls.nc != 2) return PF_EINVAL;
    OdomGPU& o = h->o;
    if (n > o.in_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(o.device));
    const int p = o.frames % kSlots;
    bool direct = false;
    int rc = host_upload(o, p, 1, &xyzi, &n, &stride_bytes, &direct);
    if (rc) return rc;
    rc = enqueue_frame(h, o.hs->d[p], n, nullptr, nullptr);
    // direct: a DMA from the caller's own pinned buffer is queued; the header lets the caller reuse the
    // buffer once this returns, so wait for that copy on the error path too
    if (direct && hipEventSynchronize(o.hs->ev[p]) != hipSuccess && !rc) rc = PF_EHIP;
    if (rc) return rc;
    if (pose_out) return read_pose(h, pose_out);
    return PF_OK;
}

int pf_bpf_frame_device(pf_odom* h, const float* d_beam, size_t nb, const float* d_pillar, size_t np,
                        const float* d_facade, size_t nf, double pose_out[7]) {
    if (!h || h->o.cls.nc != 3 || (!d_beam && nb) || (!d_pillar && np) || (!d_facade && nf)) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    const float4* cl[3] = {reinterpret_cast<const float4*>(d_beam), reinterpret_cast<const float4*>(d_pillar),
                           reinterpret_cast<const float4*>(d_facade)};
    const size_t n[3] = {nb, np, nf};
    int rc = enqueue_frame(h, nullptr, 0, cl, n);
    if (rc) return rc;
    if (pose_out) return read_pose(h, pose_out);
    return PF_OK;
}

int pf_bpf_set_front_end(pf_odom* h, const pf_cls_params* p) {
    if (!h || h->o.cls.nc != 3 || !p || p->k < 1 || p->k > kClsMaxK || !(p->radius > 0.f) || p->radius > 1.0f ||
        !(p->gf_grid_res > 0.f))
        return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    if (!o.front) {
        o.front = new ClsGPU();
        const int rc = cls_alloc(*o.front, o.in_cap);
        if (rc) {
            cls_free(*o.front);
            delete o.front;
            o.front = nullptr;
            return rc;
        }
        o.front->sticky = o.errw + E_FRONT;                     // CC_ERR latches into the handle
        alias_err(o.front->grid.err, o.errw + E_FRONT_GRID);
        if (!h->front_counted) {
            h->front_counted = true;
            g_front_handles.fetch_add(1);
        }
    }
    o.front->prm = *p;
    if (o.front2) o.front2->prm = *p;
    for (int s = 0; s < kSlots; ++s)        // parameters are baked into the captured kernels
        if (o.graph_as[s]) {
            (void)hipGraphExecDestroy(o.graph_as[s]);
            o.graph_as[s] = nullptr;
        }
    drop_graphs_f(o);
    return PF_OK;
}

int pf_bpf_set_dcvc(pf_odom* h, const pf_dcvc_params* p) {
    if (!h || h->o.cls.nc != 3) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    if (!o.front) {
        pf_cls_params fp;
        pf_cls_default_params(&fp);
        const int rc = pf_bpf_set_front_end(h, &fp);
        if (rc) return rc;
    }
    PF_HIP_TRY(odom_sync_a(o));
    const bool was_on = o.front->dcvc != nullptr;
    int rc = cls_set_dcvc(*o.front, p);
    if (!rc) o.dcvc_first = p && (!was_on || o.dcvc_first);    // a fresh instance: its first call is next
    if (!rc && o.front2) {
        const bool fresh = p && !o.front2->dcvc;
        rc = cls_set_dcvc(*o.front2, p);
        if (!rc && fresh) rc = dcvc_mark_called(*o.front2->dcvc, o.stream);
        if (!rc && fresh) PF_HIP_TRY(hipStreamSynchronize(o.stream));
    }
    if (rc) return rc;
    for (int s = 0; s < kSlots; ++s)        // the front end's kernel sequence changed
        if (o.graph_as[s]) {
            (void)hipGraphExecDestroy(o.graph_as[s]);
            o.graph_as[s] = nullptr;
        }
    drop_graphs_f(o);
    return PF_OK;
}

int pf_bpf_set_front_lanes(pf_odom* h, int lanes) {
    if (!h || h->o.cls.nc != 3 || lanes < 0 || lanes > 2) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    o.front_lanes = lanes;
    return PF_OK;
}

int pf_bpf_frame_scan_device(pf_odom* h, const float* d_xyzi, size_t n, double pose_out[7]) {
    if (!h || (!d_xyzi && n) || h->o.cls.nc != 3) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    if (!h->o.front) {
        pf_cls_params p;
        pf_cls_default_params(&p);
        const int rc = pf_bpf_set_front_end(h, &p);
        if (rc) return rc;
    }
    int rc = enqueue_frame(h, reinterpret_cast<const float4*>(d_xyzi), n, nullptr, nullptr);
    if (rc) return rc;
    // the front end's capacity flags (ground grid above its cell limit, U grid above its cell
    // capacity: the frame ran with empty class clouds) are sticky error words, reported here
    if (pose_out) return read_pose(h, pose_out);
    return PF_OK;
}

int pf_odom_set_stage_a_reserve(pf_odom* h, int cus) {
    if (!h || cus < 0) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    PF_HIP_TRY(hipStreamSynchronize(h->o.stream));
    return odom_stage_a_stream(h->o, cus);
}

int pf_odom_sync(pf_odom* h) {
    if (!h) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    PF_HIP_TRY(odom_sync_a(h->o));
    PF_HIP_TRY(hipStreamSynchronize(h->o.stream));
    PF_HIP_TRY(hipGetLastError());
    return sticky_status(h->o);
}

int pf_odom_set_stage_timing(pf_odom* h, int enable) {
    if (!h) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    PF_HIP_TRY(odom_sync_a(h->o));
    PF_HIP_TRY(hipStreamSynchronize(h->o.stream));
    if (!enable) {
        timing_free(h);
        return PF_OK;
    }
    if (!h->timing) {
        h->timing = new StageTiming();
        for (auto& q : h->timing->ev)
            for (hipEvent_t& e : q)
                if (hipEventCreate(&e) != hipSuccess) {
                    timing_free(h);
                    return PF_EHIP;
                }
    }
    StageTiming& t = *h->timing;
    for (bool& pd : t.pending) pd = false;
    t.next = 0;
    t.sum_a = t.sum_b = 0;
    t.frames = 0;
    t.on = true;
    return PF_OK;
}

int pf_odom_stage_times(pf_odom* h, double* a_us, double* b_us, size_t* frames) {
    if (!h) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    PF_HIP_TRY(odom_sync_a(h->o));
    PF_HIP_TRY(hipStreamSynchronize(h->o.stream));
    StageTiming* t = h->timing;
    if (t)
        for (int j = 0; j < StageTiming::kRing; ++j)
            if (int rc = timing_harvest(*t, j)) return rc;
    const size_t f = t ? t->frames : 0;
    if (frames) *frames = f;
    if (a_us) *a_us = f ? t->sum_a / (double)f : 0.0;
    if (b_us) *b_us = f ? t->sum_b / (double)f : 0.0;
    return PF_OK;
}

int pf_odom_poses(pf_odom* h, double* poses, size_t cap, size_t* n) {
    if (!h || !n) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    const size_t f = (size_t)o.frames;
    *n = f;
    if (!poses) return PF_OK;
    if (f > cap || f > o.pose_cap) return PF_ECAPACITY;
    if (f) {
        PF_HIP_TRY(hipMemcpyAsync(poses, o.poses, sizeof(double) * 7 * f, hipMemcpyDeviceToHost, o.stream));
        PF_HIP_TRY(hipStreamSynchronize(o.stream));
    }
    return sticky_status(o);
}

// development probe (not part of include/pfilter_hip.h): device timestamps of the last LM solve
extern "C" int pf_dev_probe(pf_odom* h, unsigned long long* out, int n) {
    if (!h || !out || n <= 0 || n > kDbgWords || !h->o.dbg) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    PF_HIP_TRY(hipStreamSynchronize(h->o.stream));
    PF_HIP_TRY(hipMemcpy(out, h->o.dbg, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
    return PF_OK;
}

int pf_odom_set_ring_model(pf_odom* h, double top_deg, double bottom_deg) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    const int rc = fe_set_ring_model(o.fe, top_deg, bottom_deg);
    if (rc) return rc;
    for (int s = 0; s < kSlots; ++s)        // the ring model is baked into the captured stage-A kernels
        if (o.graph_a[s]) {
            (void)hipGraphExecDestroy(o.graph_a[s]);
            o.graph_a[s] = nullptr;
        }
    return PF_OK;
}

// ---- state access: the public members of OdomBaseClass, snapshot / restore, map export ----------
int pf_odom_get_state(pf_odom* h, double parameters[7], double last_odom[12], int* optimization_count) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    int rc = PF_OK;
    if (o.rd_frames != o.frames) rc = readback(h);      // else: the state read with the last pose
    const DevState& st = o.h_rd->st;
    if (parameters) std::memcpy(parameters, st.params, sizeof(st.params));
    if (last_odom)
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) last_odom[4 * i + j] = st.lastR[3 * i + j];
            last_odom[4 * i + 3] = st.lastt[i];
        }
    if (optimization_count) *optimization_count = st.optimization_count;
    return rc;
}

int pf_odom_set_state(pf_odom* h, const double odom_pose[7], const double last_pose[7], int optimization_count) {
    if (!h || !odom_pose || optimization_count < 0) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    DevState st;
    PF_HIP_TRY(hipMemcpy(&st, o.st, sizeof(st), hipMemcpyDeviceToHost));
    const double* lp = last_pose ? last_pose : odom_pose;
    const pf::m3 R = pf::q2m(pf::qd{odom_pose[0], odom_pose[1], odom_pose[2], odom_pose[3]});
    const pf::m3 L = pf::q2m(pf::qd{lp[0], lp[1], lp[2], lp[3]});
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            st.odomR[3 * i + j] = R.m[i][j];
            st.lastR[3 * i + j] = L.m[i][j];
        }
        st.odomt[i] = odom_pose[4 + i];
        st.lastt[i] = lp[4 + i];
    }
    for (int k = 0; k < 7; ++k) st.params[k] = odom_pose[k];
    st.optimization_count = optimization_count;
    PF_HIP_TRY(hipMemcpy(o.st, &st, sizeof(st), hipMemcpyHostToDevice));
    o.opt_count_host = optimization_count;
    o.inited = true;                       // the next frame runs updatePointsToMap on the set maps
    o.rd_frames = -1;
    return PF_OK;
}

namespace {
// snapshot blob: header, the device state, the counters, the latest pose, then the maps
struct SnapHeader {
    uint32_t magic, version;
    int32_t nc, inited, opt_count_host, frames;
    int32_t num_lines, k_new, theta_max, weight_type;
    double map_res, min_dist, max_dist, ring_top, ring_scale;
    float theta_p;
    int32_t pad;
    uint64_t map_n[kMaxC];
};
constexpr uint32_t kSnapMagic = 0x4e534650u;   // "PFSN"
size_t snap_bytes(const SnapHeader& hd) {
    size_t b = sizeof(SnapHeader) + sizeof(DevState) + sizeof(int) * C_COUNT + sizeof(double) * 7;
    for (int c = 0; c < hd.nc; ++c) b += sizeof(float4) * hd.map_n[c];
    return b;
}
}  // namespace

int pf_odom_snapshot(pf_odom* h, void* buf, size_t cap, size_t* size) {
    if (!h || !size) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipMemcpyAsync(o.h_cnt, o.cnt, sizeof(int) * C_COUNT, hipMemcpyDeviceToHost, o.stream));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    SnapHeader hd{};
    hd.magic = kSnapMagic;
    hd.version = 1;
    hd.nc = o.cls.nc;
    hd.inited = o.inited ? 1 : 0;
    hd.opt_count_host = o.opt_count_host;
    hd.frames = o.frames;
    hd.num_lines = o.lidar.num_lines;
    hd.k_new = o.prm.k_new;
    hd.theta_max = o.prm.theta_max;
    hd.weight_type = o.prm.weight_type;
    hd.map_res = o.prm.map_res;
    hd.min_dist = o.lidar.min_dist;
    hd.max_dist = o.lidar.max_dist;
    hd.ring_top = o.fe.ring_top;
    hd.ring_scale = o.fe.ring_scale;
    hd.theta_p = o.prm.theta_p;
    for (int c = 0; c < o.cls.nc; ++c) hd.map_n[c] = (uint64_t)o.h_cnt[C_M + c];
    *size = snap_bytes(hd);
    if (!buf) return PF_OK;
    if (cap < *size) return PF_ECAPACITY;
    char* b = static_cast<char*>(buf);
    std::memcpy(b, &hd, sizeof(hd));
    b += sizeof(hd);
    PF_HIP_TRY(hipMemcpyAsync(b, o.st, sizeof(DevState), hipMemcpyDeviceToHost, o.stream));
    b += sizeof(DevState);
    std::memcpy(b, o.h_cnt, sizeof(int) * C_COUNT);
    b += sizeof(int) * C_COUNT;
    double pose[7] = {0, 0, 0, 1, 0, 0, 0};
    if (o.frames > 0)
        PF_HIP_TRY(hipMemcpyAsync(pose, o.poses + 7 * ((size_t)(o.frames - 1) % o.pose_cap), sizeof(pose),
                                  hipMemcpyDeviceToHost, o.stream));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    std::memcpy(b, pose, sizeof(pose));
    b += sizeof(pose);
    for (int c = 0; c < o.cls.nc; ++c) {
        if (hd.map_n[c])
            PF_HIP_TRY(hipMemcpyAsync(b, map_cur(o)[c], sizeof(float4) * hd.map_n[c], hipMemcpyDeviceToHost, o.stream));
        b += sizeof(float4) * hd.map_n[c];
    }
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    return sticky_status(o);
}

int pf_odom_restore(pf_odom* h, const void* buf, size_t size) {
    if (!h || !buf || size < sizeof(SnapHeader)) return PF_EINVAL;
    OdomGPU& o = h->o;
    SnapHeader hd;
    std::memcpy(&hd, buf, sizeof(hd));
    if (hd.magic != kSnapMagic || hd.version != 1 || hd.nc != o.cls.nc || size != snap_bytes(hd)) return PF_EINVAL;
    // the snapshot's estimator must be this handle's (the kernels and graphs carry its parameters)
    if (hd.num_lines != o.lidar.num_lines || hd.k_new != o.prm.k_new || hd.theta_max != o.prm.theta_max ||
        hd.weight_type != o.prm.weight_type || hd.map_res != o.prm.map_res || hd.theta_p != o.prm.theta_p ||
        hd.min_dist != o.lidar.min_dist || hd.max_dist != o.lidar.max_dist || hd.ring_top != o.fe.ring_top ||
        hd.ring_scale != o.fe.ring_scale)
        return PF_EINVAL;
    for (int c = 0; c < hd.nc; ++c)
        if (hd.map_n[c] > o.map_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(o.device));
    int rc = odom_reset(o);                    // quiesces both streams, empties the p-index buckets
    if (rc) return rc;
    const char* b = static_cast<const char*>(buf) + sizeof(hd);
    DevState st;
    std::memcpy(&st, b, sizeof(st));
    b += sizeof(st);
    int cnt[C_COUNT];
    std::memcpy(cnt, b, sizeof(cnt));
    b += sizeof(cnt);
    double pose[7];
    std::memcpy(pose, b, sizeof(pose));
    b += sizeof(pose);
    // the restored handle's pose history starts with the snapshot's pose
    const bool has_pose = hd.frames > 0;
    st.frame = has_pose ? 1 : 0;
    PF_HIP_TRY(hipMemcpyAsync(o.st, &st, sizeof(st), hipMemcpyHostToDevice, o.stream));
    PF_HIP_TRY(hipMemcpyAsync(o.cnt, cnt, sizeof(cnt), hipMemcpyHostToDevice, o.stream));
    if (has_pose) PF_HIP_TRY(hipMemcpyAsync(o.poses, pose, sizeof(pose), hipMemcpyHostToDevice, o.stream));
    for (int c = 0; c < hd.nc; ++c) {
        if (hd.map_n[c])
            PF_HIP_TRY(hipMemcpyAsync(map_cur(o)[c], b, sizeof(float4) * hd.map_n[c], hipMemcpyHostToDevice, o.stream));
        b += sizeof(float4) * hd.map_n[c];
    }
    odom_dep_dirty(o, o.stream);               // the snapshot's maps: checked as host-written ones
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    o.inited = hd.inited != 0;
    o.opt_count_host = hd.opt_count_host;
    o.frames = has_pose ? 1 : 0;
    o.rd_frames = -1;
    return PF_OK;
}

int pf_odom_set_map_export(pf_odom* h, int enable) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    if (enable && !o.h_map[0]) {
        for (int c = 0; c < o.cls.nc; ++c) {
            if (hipHostMalloc(&o.h_map[c], sizeof(float4) * o.map_cap, hipHostMallocMapped) != hipSuccess)
                return PF_ENOMEM;
            PF_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&o.h_map_dev[c]), o.h_map[c], 0));
        }
        if (hipHostMalloc(&o.h_map_n, sizeof(int) * kMaxC, hipHostMallocMapped) != hipSuccess) return PF_ENOMEM;
        PF_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&o.h_map_n_dev), o.h_map_n, 0));
        std::memset(o.h_map_n, 0, sizeof(int) * kMaxC);
    }
    if ((enable != 0) != o.export_maps)
        drop_graphs_b(o);                      // the export kernel is part of the captured stage B
    o.export_maps = enable != 0;
    return PF_OK;
}

int pf_odom_map_export(pf_odom* h, int which, const float** xyzw, size_t* n) {
    if (!h || !xyzw || !n || which < 0 || which >= h->o.cls.nc || !h->o.export_maps) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));     // (already idle after a call that read the pose)
    *xyzw = reinterpret_cast<const float*>(o.h_map[which]);
    *n = (size_t)o.h_map_n[which];
    return PF_OK;
}

// development probe (not part of include/pfilter_hip.h): the sticky error words at their last report
extern "C" int pf_dev_errors(pf_odom* h, int* out, int n) {
    if (!h || !out || n <= 0 || n > E_COUNT) return PF_EINVAL;
    for (int k = 0; k < n; ++k) out[k] = h->o.err_last[k];
    return PF_OK;
}

int pf_odom_set_tie_order(pf_odom* h, int enable) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    if (enable && !o.tie_a) {
        // all or nothing: a failed allocation leaves neither sort behind, so the handle stays in the
        // stable order and a later call starts from scratch
        auto drop = [&o]() {
            for (TieSort** t : {&o.tie_a, &o.tie_b})
                if (*t) {
                    tie_free(**t);
                    delete *t;
                    *t = nullptr;
                }
        };
        o.tie_a = new (std::nothrow) TieSort();
        o.tie_b = new (std::nothrow) TieSort();
        int rc = (!o.tie_a || !o.tie_b) ? PF_ENOMEM : tie_alloc(*o.tie_a, (size_t)o.cls.nc * o.in_cap);
        if (rc == PF_OK) rc = tie_alloc(*o.tie_b, o.sort_cap);
        if (rc != PF_OK) {
            drop();
            return rc;
        }
    }
    if (enable) {
        if (int rc = odom_dep_alloc(o)) return rc;
        if (!o.tie_order) {                             // maps written by the other order's rgbds
            odom_dep_dirty(o, o.stream);
            PF_HIP_TRY(hipStreamSynchronize(o.stream));
        }
    }
    if ((enable != 0) != o.tie_order) {             // both stages' captured kernel sequences change
        for (int s = 0; s < kSlots; ++s)
            for (hipGraphExec_t* g : {&o.graph_a[s], &o.graph_as[s]})
                if (*g) {
                    (void)hipGraphExecDestroy(*g);
                    *g = nullptr;
                }
        drop_graphs_f(o);
        drop_graphs_b(o);
    }
    o.tie_order = enable != 0;
    o.fe.tie_order = o.tie_order;                   // featureExtraction's sector sort (:101-104)
    return PF_OK;
}

// development / test switch (not part of include/pfilter_hip.h): rgbds in the default order by the
// full radix sort of every element (the path before the merge) instead of the merge, for A/B checks
// development / test switch (not part of include/pfilter_hip.h): the rgbds tie sort's partition-tier
// depth-limit segments heap-sorted on stage B's side stream beside k_tie_local (1) or after
// it on stage B's own stream (0, the default), for A/B checks (TieAux, pf_tie.h)
extern "C" int pf_dev_set_tie_aux(pf_odom* h, int enable) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    if ((enable != 0) != o.tie_aux) drop_graphs_b(o);   // the captured stage B gains / loses the fork
    o.tie_aux = enable != 0;
    return PF_OK;
}

// development / test switch: every tie-order rgbds takes the full dependence table (DepTab in pf_odom.hip:
// each update starts as if the host had written the map), for the A/B check of the small table
extern "C" int pf_dev_set_dep_full(pf_odom* h, int enable) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    if ((enable != 0) != o.dep_force_full) drop_graphs_b(o);   // the captured stage B gains / loses a launch
    o.dep_force_full = enable != 0;
    return PF_OK;
}

// development: the dependence flags of the last tie-order rgbds (one byte per element, cnt[C_NRG] of them)
extern "C" int pf_dev_dep_flags(pf_odom* h, uint8_t* out, size_t cap, int* n) {
    if (!h || !out || !n) return PF_EINVAL;
    OdomGPU& o = h->o;
    if (!o.dep_free) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    int c[C_COUNT];
    PF_HIP_TRY(hipMemcpy(c, o.cnt, sizeof(c), hipMemcpyDeviceToHost));
    *n = c[C_NRG];
    if ((size_t)c[C_NRG] > cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipMemcpy(out, o.dep_free, (size_t)c[C_NRG], hipMemcpyDeviceToHost));
    return PF_OK;
}

// development: the separate k_observe launch at weightType 0 too (the path before the fused observe)
extern "C" int pf_dev_set_fuse_observe(pf_odom* h, int enable) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    if ((enable == 0) != o.no_fuse_obs) drop_graphs_b(o);
    o.no_fuse_obs = enable == 0;
    return PF_OK;
}

extern "C" int pf_dev_set_rg_radix(pf_odom* h, int enable) {
    if (!h) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    if ((enable != 0) != o.rg_radix) drop_graphs_b(o);
    o.rg_radix = enable != 0;
    return PF_OK;
}

// development / test probe (not part of include/pfilter_hip.h): the reference-tie-order sort alone on
// n host keys (bits 30-31 the class, classes back to back as the pipeline's batches hold them,
// 0xFFFFFFFF dropped anywhere); perm receives the vals (input indices) of the kept pairs in std::sort's
// order, *n_out their count. PF_EINVAL when the valid keys are not class-major.
// depth >= 0 replaces the depth limit 2 lg n of every class (the heap-sort branch, against the oracle's
// settable-depth restatement), levels = the big levels run before the medium workgroups (0: none).
extern "C" int pf_dev_tie_sort2(int device, const uint32_t* keys, size_t n, int depth, int levels, uint32_t* perm,
                                size_t* n_out) {
    if ((!keys && n) || !perm || !n_out || n > (size_t)INT_MAX / 2 || levels < 0 || levels > kMaxBigLevels) return PF_EINVAL;
    int sizes[4] = {0, 0, 0, 0};
    {
        int end[4] = {0, 0, 0, 0};                 // one past the last valid key of class <= c
        int prev = 0;
        for (size_t i = 0; i < n; ++i) {
            if (keys[i] == 0xFFFFFFFFu) continue;
            const int c = (int)(keys[i] >> 30);
            if (c < prev) return PF_EINVAL;
            prev = c;
            for (int q = c; q < 4; ++q) end[q] = (int)i + 1;
        }
        end[3] = (int)n;
        for (int c = 0; c < 4; ++c) sizes[c] = end[c] - (c ? end[c - 1] : 0);
    }
    PF_HIP_TRY(hipSetDevice(device));
    const size_t cap = n ? n : 1;
    TieSort t;
    u32 *dk = nullptr, *dv = nullptr;
    int* dsz = nullptr;
    hipStream_t s = nullptr;
    int rc = tie_alloc(t, cap, levels);
    t.depth0 = depth;
    if (!rc && (hipMalloc(&dk, sizeof(u32) * cap) != hipSuccess || hipMalloc(&dv, sizeof(u32) * cap) != hipSuccess ||
                hipMalloc(&dsz, sizeof(int) * 8) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess))
        rc = PF_ENOMEM;
    std::vector<u32> iota(cap);
    for (size_t i = 0; i < cap; ++i) iota[i] = (u32)i;
    int hsz[8] = {sizes[0], sizes[1], sizes[2], sizes[3], 0, 0, 0, 0};
    if (!rc && (hipMemcpyAsync(dk, keys, sizeof(u32) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipMemcpyAsync(dv, iota.data(), sizeof(u32) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipMemcpyAsync(dsz, hsz, sizeof(hsz), hipMemcpyHostToDevice, s) != hipSuccess))
        rc = PF_EHIP;
    // the radix route beside the tiers (TieAux::hs) as stage B runs it; PF_TIE_HS=0: on s (both tested)
    hipStream_t hs = nullptr;
    hipEvent_t evf = nullptr, evj = nullptr;
    const char* hse = std::getenv("PF_TIE_HS");
    if (!rc && levels > 0 && !(hse && std::atoi(hse) == 0) &&
        (hipStreamCreateWithFlags(&hs, hipStreamNonBlocking) != hipSuccess ||
         hipEventCreateWithFlags(&evf, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&evj, hipEventDisableTiming) != hipSuccess))
        rc = PF_EHIP;
    if (!rc) {
        TieAux aux;
        aux.fork = evf;
        aux.join = evj;
        aux.hs = hs;
        tie_sort(t, dk, dv, TieClasses{dsz, 0, -1, 4}, dsz + 4, s, levels, nullptr, hs ? &aux : nullptr);
        int nv = 0, err = 0;
        if (hipMemcpyAsync(&nv, tie_valid_count(t), sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(&err, dsz + 4, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            rc = PF_EHIP;
        else {
            *n_out = (size_t)nv;
            if (err) rc = PF_EHIP;
            else if (nv && (hipMemcpy(perm, dv, sizeof(u32) * (size_t)nv, hipMemcpyDeviceToHost) != hipSuccess)) rc = PF_EHIP;
        }
    }
    if (s) (void)hipStreamSynchronize(s);
    (void)hipFree(dk);
    (void)hipFree(dv);
    (void)hipFree(dsz);
    if (s) (void)hipStreamDestroy(s);
    if (hs) (void)hipStreamSynchronize(hs);
    if (hs) (void)hipStreamDestroy(hs);
    if (evf) (void)hipEventDestroy(evf);
    if (evj) (void)hipEventDestroy(evj);
    tie_free(t);
    return rc;
}
extern "C" int pf_dev_tie_sort(int device, const uint32_t* keys, size_t n, uint32_t* perm, size_t* n_out) {
    return pf_dev_tie_sort2(device, keys, n, -1, 2, perm, n_out);
}

int pf_odom_probe_assoc(pf_odom* h, int iters, double* avg_ms, double* alg_bytes, size_t* nq, float* queries,
                        size_t cap) {
    if (!h || !avg_ms || !alg_bytes || !nq) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->o.device));
    int n = 0;
    const int rc = odom_probe_assoc(h->o, iters, avg_ms, alg_bytes, &n, reinterpret_cast<float4*>(queries), cap);
    *nq = (size_t)(n > 0 ? n : 0);
    return rc;
}

int pf_odom_merge_stats(pf_odom* h, int* full_sorts, int* max_appended) {
    if (!h || !full_sorts || !max_appended) return PF_EINVAL;
    OdomGPU& o = h->o;
    PF_HIP_TRY(hipSetDevice(o.device));
    PF_HIP_TRY(odom_sync_a(o));
    PF_HIP_TRY(hipStreamSynchronize(o.stream));
    int st[4];
    PF_HIP_TRY(hipMemcpy(st, o.rgm_stat, sizeof(st), hipMemcpyDeviceToHost));
    *full_sorts = st[1];
    *max_appended = st[2];
    return PF_OK;
}

int pf_odom_set_graph(pf_odom* h, int mode) {
    if (!h || !(mode == PF_GRAPH_AUTO || (mode & ~(PF_GRAPH_STAGE_A | PF_GRAPH_STAGE_B)) == 0)) return PF_EINVAL;
    h->o.graph_mode = mode;
    return PF_OK;
}

// ------------------------------------------------------------------------------------------------
int pf_device_count(int* n) {
    if (!n) return PF_EINVAL;
    PF_HIP_TRY(hipGetDeviceCount(n));
    return PF_OK;
}

int pf_dev_malloc(int device, size_t bytes, void** d) {
    if (!d) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(device));
    if (hipMalloc(d, bytes) != hipSuccess) return PF_ENOMEM;
    return PF_OK;
}

int pf_dev_free(int device, void* d) {
    PF_HIP_TRY(hipSetDevice(device));
    PF_HIP_TRY(hipFree(d));
    return PF_OK;
}

int pf_host_alloc(size_t bytes, void** p) {
    if (!p || !bytes) return PF_EINVAL;
    *p = nullptr;
    void* h = nullptr;
    if (hipHostMalloc(&h, bytes, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess) return PF_ENOMEM;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return PF_EHIP;
    }
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        g_pinned[(uintptr_t)h] = PinnedBlock{bytes, static_cast<char*>(d)};
    }
    *p = h;
    return PF_OK;
}

int pf_host_free(void* p) {
    if (!p) return PF_OK;
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        if (!g_pinned.erase((uintptr_t)p)) return PF_EINVAL;
    }
    PF_HIP_TRY(hipHostFree(p));
    return PF_OK;
}

int pf_memcpy_h2d(int device, void* dst, const void* src, size_t bytes) {
    PF_HIP_TRY(hipSetDevice(device));
    PF_HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return PF_OK;
}

int pf_memcpy_d2h(int device, void* dst, const void* src, size_t bytes) {
    PF_HIP_TRY(hipSetDevice(device));
    PF_HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return PF_OK;
}

}  // extern "C"
