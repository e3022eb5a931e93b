// pfref: Odom_ES_EstimationClass + third-party semantics restated.
// TEST INFRASTRUCTURE (oracle) — see pfref.h header.
#include "pfref_internal.h"

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <array>
#include <map>
#include <memory>

namespace pfref {

// ------------------------------------------------------------------------------------------
// PCL 1.10 VoxelGrid<PointXYZRGB>::applyFilter, downsample_all_data_ = true
// ------------------------------------------------------------------------------------------
thread_local bool g_ld_trig = false;
thread_local bool g_qr_rev = false;
thread_local bool g_quad = false;      // PFREF_LM_QUAD (experiment)
thread_local bool g_cost_rev = false;  // PFREF_COST_REVSUM (experiment)
thread_local bool g_dev_libm = false;  // PFREF_DEV_LIBM (experiment)
thread_local bool g_dev_half = false;  // PFREF_DEV_HALFANGLE (experiment)

// development: PFREF_TRIG_DUMP=<file> appends every libm argument of the faithful LM (doubles)
void trig_dump(double v) {
    static FILE* f = std::getenv("PFREF_TRIG_DUMP") ? std::fopen(std::getenv("PFREF_TRIG_DUMP"), "ab") : nullptr;
    if (f) std::fwrite(&v, sizeof(v), 1, f);
}

namespace {
struct IdxPair { unsigned idx, cloud_point_index; };

void minmax3(const std::vector<PtC>& in, float mn[3], float mx[3]) {  // pcl::getMinMax3D
    for (int d = 0; d < 3; ++d) { mn[d] = FLT_MAX; mx[d] = -FLT_MAX; }
    for (const PtC& p : in) {
        const float v[3] = {p.x, p.y, p.z};
        for (int d = 0; d < 3; ++d) { mn[d] = std::min(mn[d], v[d]); mx[d] = std::max(mx[d], v[d]); }
    }
}

void sort_pairs(std::vector<IdxPair>& iv, bool stable) {
    auto lt = [](const IdxPair& a, const IdxPair& b) { return a.idx < b.idx; };
    static const bool trace = std::getenv("PFREF_SORT_STATS") != nullptr;   // development statistics
    if (trace && !stable) {
        std::vector<uint32_t> k(iv.size());
        for (size_t i = 0; i < iv.size(); ++i) k[i] = iv[i].idx;
        long st[7];
        pfref_introsort_stats(k.data(), k.size(), st);
        std::fprintf(stderr, "sort n %zu levels %ld heaps %ld max %ld keys %ld g3segs %ld g3max %ld dupkeys %ld\n", k.size(),
                     st[0], st[1], st[2], st[3], st[4], st[5], st[6]);
        if (const char* dump = std::getenv("PFREF_SORT_DUMP")) {   // keys of sorts above PFREF_SORT_DUMP_MIN
            static const size_t dmin = std::getenv("PFREF_SORT_DUMP_MIN") ?     // (default 1M), appended,
                std::strtoull(std::getenv("PFREF_SORT_DUMP_MIN"), nullptr, 10) : (1u << 20);   // each after its count
            if (k.size() > dmin) {
                if (FILE* f = std::fopen(dump, "ab")) {
                    const uint32_t cnt = (uint32_t)k.size();
                    if (dmin != (1u << 20)) std::fwrite(&cnt, sizeof(cnt), 1, f);
                    std::fwrite(k.data(), sizeof(uint32_t), k.size(), f);
                    std::fclose(f);
                }
            }
        }
    }
    if (stable) std::stable_sort(iv.begin(), iv.end(), lt);
    else std::sort(iv.begin(), iv.end(), lt);
}

// development statistics (PFREF_GROUP_STATS): of one sorted call, the voxel groups whose f32 centroid
// sum depends on the order of their points. A group of <= 2 is order-free (0 + a is exact, + commutes);
// a group of 3 has three left folds, compared per coordinate; 4 and more count as order-dependent.
void group_stats(const char* what, const std::vector<PtC>& in, const std::vector<IdxPair>& iv) {
    static const bool on = std::getenv("PFREF_GROUP_STATS") != nullptr;
    if (!on) return;
    long g[4] = {0, 0, 0, 0}, dep3 = 0, gmax = 0, dep_keys = 0;
    std::vector<uint32_t> keys(iv.size());
    std::vector<uint8_t> depf(iv.size(), 0);
    for (const IdxPair& q : iv) keys[q.cloud_point_index] = q.idx;
    size_t index = 0;
    while (index < iv.size()) {
        size_t i = index + 1;
        while (i < iv.size() && iv[i].idx == iv[index].idx) ++i;
        const long n = (long)(i - index);
        gmax = std::max(gmax, n);
        ++g[std::min(n, 4L) - 1];
        if (n == 3) {
            const PtC& a = in[iv[index].cloud_point_index];
            const PtC& b = in[iv[index + 1].cloud_point_index];
            const PtC& c = in[iv[index + 2].cloud_point_index];
            bool dep = false;
            const float va[3] = {a.x, a.y, a.z}, vb[3] = {b.x, b.y, b.z}, vc[3] = {c.x, c.y, c.z};
            for (int d = 0; d < 3; ++d) {
                volatile float f1 = (va[d] + vb[d]) + vc[d], f2 = (va[d] + vc[d]) + vb[d], f3 = (vb[d] + vc[d]) + va[d];
                dep |= !(f1 == f2 && f1 == f3);
            }
            dep3 += dep;
            if (dep) dep_keys += 3;
            if (dep)
                for (size_t li = index; li < i; ++li) depf[iv[li].cloud_point_index] = 1;
        } else if (n >= 4) {
            dep_keys += n;
            for (size_t li = index; li < i; ++li) depf[iv[li].cloud_point_index] = 1;
        }
        index = i;
    }
    pfref_introsort_heapdep(keys.data(), depf.data(), keys.size(), what);
    std::fprintf(stderr, "groups %s n %zu g1 %ld g2 %ld g3 %ld dep3 %ld g4+ %ld max %ld depkeys %ld\n", what, iv.size(),
                 g[0], g[1], g[2], dep3, g[3], gmax, dep_keys);
}
}  // namespace

void voxel_grid(const std::vector<PtC>& in, float leaf, bool stable, std::vector<PtC>& out) {
    out.clear();
    if (in.empty()) return;
    const float inv = 1.0f / leaf;  // inverse_leaf_size_ = Array4f::Ones() / leaf_size_
    float mn[3], mx[3];
    minmax3(in, mn, mx);
    int64_t dx = static_cast<int64_t>((mx[0] - mn[0]) * inv) + 1;
    int64_t dy = static_cast<int64_t>((mx[1] - mn[1]) * inv) + 1;
    int64_t dz = static_cast<int64_t>((mx[2] - mn[2]) * inv) + 1;
    if ((dx * dy * dz) > static_cast<int64_t>(INT32_MAX)) {  // "Leaf size is too small": copy input
        out = in;
        return;
    }
    int min_b[3], max_b[3], div_b[3], mul[3];
    for (int d = 0; d < 3; ++d) {
        min_b[d] = static_cast<int>(std::floor(mn[d] * inv));
        max_b[d] = static_cast<int>(std::floor(mx[d] * inv));
        div_b[d] = max_b[d] - min_b[d] + 1;
    }
    mul[0] = 1; mul[1] = div_b[0]; mul[2] = div_b[0] * div_b[1];
    std::vector<IdxPair> iv;
    iv.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        const PtC& p = in[i];
        int i0 = static_cast<int>(std::floor(p.x * inv) - static_cast<float>(min_b[0]));
        int i1 = static_cast<int>(std::floor(p.y * inv) - static_cast<float>(min_b[1]));
        int i2 = static_cast<int>(std::floor(p.z * inv) - static_cast<float>(min_b[2]));
        int idx = i0 * mul[0] + i1 * mul[1] + i2 * mul[2];
        iv.push_back({static_cast<unsigned>(idx), static_cast<unsigned>(i)});
    }
    sort_pairs(iv, stable);
    group_stats("vg", in, iv);
    size_t index = 0;
    while (index < iv.size()) {
        size_t i = index + 1;
        while (i < iv.size() && iv[i].idx == iv[index].idx) ++i;
        // CentroidPoint<PointXYZRGB>: AccumulatorXYZ (Vector3f sum) + AccumulatorRGBA (float sums)
        float sx = 0, sy = 0, sz = 0, sr = 0, sg = 0, sb = 0;
        for (size_t li = index; li < i; ++li) {
            const PtC& p = in[iv[li].cloud_point_index];
            sx += p.x; sy += p.y; sz += p.z;
            sr += static_cast<float>(p.r); sg += static_cast<float>(p.g); sb += static_cast<float>(p.b);
        }
        const size_t n = i - index;
        PtC o;
        o.x = sx / n; o.y = sy / n; o.z = sz / n;
        o.r = static_cast<uint8_t>(static_cast<uint32_t>(sr / n));
        o.g = static_cast<uint8_t>(static_cast<uint32_t>(sg / n));
        o.b = static_cast<uint8_t>(static_cast<uint32_t>(sb / n));
        out.push_back(o);
        index = i;
    }
}

// OdomBaseClass::rgbds (src/odomEstimationClass.cpp:34-134)
void rgbds(const std::vector<PtC>& in, float dsleaf, bool stable, std::vector<PtC>& out) {
    out.clear();
    if (in.empty()) return;
    float mn[3], mx[3];
    minmax3(in, mn, mx);
    int min_b[3], max_b[3], div_b[3], mul[3];
    for (int d = 0; d < 3; ++d) {                                   // :46-51 (f32 division)
        min_b[d] = static_cast<int>(std::floor(mn[d] / dsleaf));
        max_b[d] = static_cast<int>(std::floor(mx[d] / dsleaf));
        div_b[d] = max_b[d] - min_b[d] + 1;
    }
    mul[0] = 1; mul[1] = div_b[0]; mul[2] = div_b[0] * div_b[1];
    std::vector<IdxPair> iv;
    iv.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {                       // :61-70
        const PtC& p = in[i];
        int i0 = static_cast<int>(std::floor(p.x / dsleaf) - static_cast<float>(min_b[0]));
        int i1 = static_cast<int>(std::floor(p.y / dsleaf) - static_cast<float>(min_b[1]));
        int i2 = static_cast<int>(std::floor(p.z / dsleaf) - static_cast<float>(min_b[2]));
        int idx = i0 * mul[0] + i1 * mul[1] + i2 * mul[2];
        iv.push_back({static_cast<unsigned>(idx), static_cast<unsigned>(i)});
    }
    sort_pairs(iv, stable);                                        // :74
    group_stats("rg", in, iv);
    size_t index = 0;
    while (index < iv.size()) {                                    // :86-131
        size_t i = index + 1;
        while (i < iv.size() && iv[i].idx == iv[index].idx) ++i;
        float cx = 0, cy = 0, cz = 0;  // Vector4f centroid (w lane is 1/n * n = 1, unused)
        int r_max = -1;
        float g_max = -1;
        for (size_t li = index; li < i; ++li) {
            const PtC& p = in[iv[li].cloud_point_index];
            cx += p.x; cy += p.y; cz += p.z;
            if (p.r > r_max) r_max = p.r;
            if (p.g > g_max) g_max = p.g;
        }
        const float n = static_cast<float>(i - index);
        PtC o;
        o.x = cx / n; o.y = cy / n; o.z = cz / n;
        o.r = static_cast<uint8_t>(r_max);
        o.g = static_cast<uint8_t>(g_max);
        o.b = 0;
        out.push_back(o);
        index = i;
    }
}

// ------------------------------------------------------------------------------------------
// kNN: FLANN 1.9.1 KDTreeSingleIndex-style tree (leaf 15, middle split) with an exact
// (d2, index)-ordered result set; brute force for cross-checks.
// ------------------------------------------------------------------------------------------
struct KnnSet {
    int k, count = 0;
    float d[8];
    int id[8];
    explicit KnnSet(int kk) : k(kk) {}
    bool full() const { return count == k; }
    float worst() const { return full() ? d[k - 1] : FLT_MAX; }
    void add(float dist, int index) {
        if (full() && (dist > d[k - 1] || (dist == d[k - 1] && index >= id[k - 1]))) return;
        int i = full() ? k - 1 : count++;
        while (i > 0 && (d[i - 1] > dist || (d[i - 1] == dist && id[i - 1] > index))) {
            d[i] = d[i - 1]; id[i] = id[i - 1]; --i;
        }
        d[i] = dist; id[i] = index;
    }
};

void knn_brute(const std::vector<PtC>& map, const float q[3], int k, int* idx, float* d2) {
    KnnSet rs(k);
    for (size_t i = 0; i < map.size(); ++i) {
        const float p[3] = {map[i].x, map[i].y, map[i].z};
        rs.add(l2f(q, p), (int)i);
    }
    for (int j = 0; j < k; ++j) {
        idx[j] = j < rs.count ? rs.id[j] : -1;
        d2[j] = j < rs.count ? rs.d[j] : FLT_MAX;
    }
}

void KdTree::build(const std::vector<PtC>& pts) {
    const size_t n = pts.size();
    xyz_.resize(3 * n);
    vind_.resize(n);
    for (size_t i = 0; i < n; ++i) vind_[i] = (int)i;
    nodes_.clear();
    nodes_.reserve(2 * (n / 8 + 1));
    std::vector<float> raw(3 * n);
    for (size_t i = 0; i < n; ++i) { raw[3 * i] = pts[i].x; raw[3 * i + 1] = pts[i].y; raw[3 * i + 2] = pts[i].z; }
    xyz_.swap(raw);  // temporarily indexed by original id during the build
    if (n == 0) { root_ = -1; return; }
    float bmin[3], bmax[3];
    for (int d = 0; d < 3; ++d) { bmin[d] = FLT_MAX; bmax[d] = -FLT_MAX; }
    for (size_t i = 0; i < n; ++i)
        for (int d = 0; d < 3; ++d) { bmin[d] = std::min(bmin[d], xyz_[3 * i + d]); bmax[d] = std::max(bmax[d], xyz_[3 * i + d]); }
    root_ = build_rec(0, (int)n, bmin, bmax);
    // reorder the dataset (FLANN reorder_ = true)
    std::vector<float> re(3 * n);
    for (size_t i = 0; i < n; ++i)
        for (int d = 0; d < 3; ++d) re[3 * i + d] = xyz_[3 * (size_t)vind_[i] + d];
    xyz_.swap(re);
}

int KdTree::build_rec(int lo, int hi, const float* bmin, const float* bmax) {
    Node node{};
    node.left = lo; node.right = hi; node.child1 = node.child2 = -1;
    int me = (int)nodes_.size();
    nodes_.push_back(node);
    if (hi - lo <= 15) return me;
    float max_span = -1;
    for (int d = 0; d < 3; ++d) max_span = std::max(max_span, bmax[d] - bmin[d]);
    int cutfeat = 0;
    float max_spread = -1;
    for (int d = 0; d < 3; ++d) {
        if (bmax[d] - bmin[d] > (1 - 0.00001f) * max_span) {
            float mn = FLT_MAX, mx = -FLT_MAX;
            for (int i = lo; i < hi; ++i) { float v = xyz_[3 * (size_t)vind_[i] + d]; mn = std::min(mn, v); mx = std::max(mx, v); }
            if (mx - mn > max_spread) { max_spread = mx - mn; cutfeat = d; }
        }
    }
    float mn = FLT_MAX, mx = -FLT_MAX;
    for (int i = lo; i < hi; ++i) { float v = xyz_[3 * (size_t)vind_[i] + cutfeat]; mn = std::min(mn, v); mx = std::max(mx, v); }
    float split = (bmin[cutfeat] + bmax[cutfeat]) / 2;
    float cutval = split < mn ? mn : (split > mx ? mx : split);
    // planeSplit: [< cutval | == cutval | > cutval]
    int l = lo, r = hi - 1;
    while (l <= r) {
        while (l <= r && xyz_[3 * (size_t)vind_[l] + cutfeat] < cutval) ++l;
        while (l <= r && xyz_[3 * (size_t)vind_[r] + cutfeat] >= cutval) --r;
        if (l < r) std::swap(vind_[l], vind_[r]);
    }
    int lim1 = l - lo;
    r = hi - 1;
    while (l <= r) {
        while (l <= r && xyz_[3 * (size_t)vind_[l] + cutfeat] <= cutval) ++l;
        while (l <= r && xyz_[3 * (size_t)vind_[r] + cutfeat] > cutval) --r;
        if (l < r) std::swap(vind_[l], vind_[r]);
    }
    int lim2 = l - lo;
    int count = hi - lo, index;
    if (lim1 > count / 2) index = lim1;
    else if (lim2 < count / 2) index = lim2;
    else index = count / 2;
    if (index == 0 || index == count) index = count / 2;  // degenerate (all equal): plain halving
    float lmax[3], rmin[3];
    std::copy(bmax, bmax + 3, lmax); lmax[cutfeat] = cutval;
    std::copy(bmin, bmin + 3, rmin); rmin[cutfeat] = cutval;
    int c1 = build_rec(lo, lo + index, bmin, lmax);
    int c2 = build_rec(lo + index, hi, rmin, bmax);
    // tight split bounds along cutfeat
    float dl = -FLT_MAX, dh = FLT_MAX;
    for (int i = lo; i < lo + index; ++i) dl = std::max(dl, xyz_[3 * (size_t)vind_[i] + cutfeat]);
    for (int i = lo + index; i < hi; ++i) dh = std::min(dh, xyz_[3 * (size_t)vind_[i] + cutfeat]);
    nodes_[me].divfeat = cutfeat;
    nodes_[me].divlow = dl;
    nodes_[me].divhigh = dh;
    nodes_[me].child1 = c1;
    nodes_[me].child2 = c2;
    return me;
}

void KdTree::search(int ni, const float q[3], float mindist, float dists[3], KnnSet& rs) const {
    const Node& nd = nodes_[ni];
    if (nd.child1 < 0) {
        for (int i = nd.left; i < nd.right; ++i) rs.add(l2f(q, &xyz_[3 * (size_t)i]), vind_[i]);
        return;
    }
    const int f = nd.divfeat;
    const float val = q[f];
    const float diff1 = val - nd.divlow, diff2 = val - nd.divhigh;
    int best, other;
    float cut;
    if ((diff1 + diff2) < 0) { best = nd.child1; other = nd.child2; cut = diff2 * diff2; }
    else { best = nd.child2; other = nd.child1; cut = diff1 * diff1; }
    search(best, q, mindist, dists, rs);
    float dst = dists[f];
    float md = mindist + cut - dst;
    dists[f] = cut;
    // <= with a relative slack: the float bound may round above an equal-distance point
    if (md * (1.0f - 1e-5f) <= rs.worst()) search(other, q, md, dists, rs);
    dists[f] = dst;
}

int KdTree::knn(const float q[3], int k, int* idx, float* d2) const {
    KnnSet rs(k);
    if (root_ >= 0) {
        float dists[3] = {0, 0, 0};
        search(root_, q, 0.0f, dists, rs);
    }
    for (int j = 0; j < k; ++j) {
        idx[j] = j < rs.count ? rs.id[j] : -1;
        d2[j] = j < rs.count ? rs.d[j] : FLT_MAX;
    }
    return rs.count;
}

// ------------------------------------------------------------------------------------------
// Ceres 1.14 Solve emulation for one SE(3) parameter block
// ------------------------------------------------------------------------------------------
struct Residual {
    bool edge;
    V3 cur, a, b;   // edge: line points; surf: a = unit normal
    double d;       // surf: (double)(float)negative_OA_dot_norm
    double w;       // point_weight (0 = none)
    int q;          // index of the query in the classes' concatenated down-sampled clouds
};

namespace {
const double kHuberA = 0.1;
const double kHuberB = 0.1 * 0.1;

// evaluates corrected residuals/Jacobians (HuberLoss + Corrector); returns false if non-finite
bool evaluate(const std::vector<Residual>& res, const double* x, double& cost, std::vector<double>* r,
              std::vector<double>* J) {
    cost = 0.0;
    static thread_local std::vector<double> hc;
    if (g_cost_rev) hc.assign(res.size(), 0.0);
    for (size_t i = 0; i < res.size(); ++i) {
        const Residual& q = res[i];
        double Jl[7];
        double ri = q.edge ? edge_eval(x, q.cur, q.a, q.b, q.w, J ? Jl : nullptr)
                           : surf_eval(x, q.cur, q.a, q.d, q.w, J ? Jl : nullptr);
        if (!std::isfinite(ri)) return false;
        if (J) for (int j = 0; j < 6; ++j) if (!std::isfinite(Jl[j])) return false;
        double s = ri * ri;
        double rho0, rho1;
        if (s > kHuberB) {
            double rr = std::sqrt(s);
            rho0 = 2.0 * kHuberA * rr - kHuberB;
            rho1 = std::max(std::numeric_limits<double>::min(), kHuberA / rr);
        } else {
            rho0 = s; rho1 = 1.0;
        }
        if (g_cost_rev) hc[i] = 0.5 * rho0;
        else cost += 0.5 * rho0;
        double srho1 = std::sqrt(rho1);
        if (J) for (int j = 0; j < 6; ++j) (*J)[6 * i + j] = Jl[j] * srho1;
        if (r) (*r)[i] = ri * srho1;
    }
    if (g_cost_rev)
        for (size_t i = res.size(); i-- > 0;) cost += hc[i];
    return true;
}

// Eigen HouseholderQR (unblocked) solve of the (m+6) x 6 augmented system, column-major A.
void householder_solve(std::vector<double>& A, int rows, int cols, std::vector<double>& rhs, double* x) {
    std::vector<double> hc(cols);
    auto at = [&](int i, int j) -> double& { return A[(size_t)j * rows + i]; };
    std::vector<double> xx(rows), ess(rows);
    for (int k = 0; k < cols; ++k) {
        int n = rows - k;
        for (int i = 0; i < n; ++i) xx[i] = at(k + i, k);
        double tau, beta;
        make_householder(xx.data(), n, ess.data(), tau, beta);
        at(k, k) = beta;
        for (int i = 1; i < n; ++i) at(k + i, k) = ess[i];
        hc[k] = tau;
        if (tau != 0.0 && n > 1) {
            for (int j = k + 1; j < cols; ++j) {
                double tmp = 0.0;
                if (g_qr_rev)
                    for (int i = n - 1; i >= 1; --i) tmp += ess[i] * at(k + i, j);
                else
                    for (int i = 1; i < n; ++i) tmp += ess[i] * at(k + i, j);
                tmp += at(k, j);
                at(k, j) -= tau * tmp;
                for (int i = 1; i < n; ++i) at(k + i, j) -= tau * ess[i] * tmp;
            }
        }
    }
    for (int k = 0; k < cols; ++k) {
        int n = rows - k;
        if (hc[k] == 0.0 || n < 2) continue;
        double tmp = 0.0;
        if (g_qr_rev)
            for (int i = n - 1; i >= 1; --i) tmp += at(k + i, k) * rhs[k + i];
        else
            for (int i = 1; i < n; ++i) tmp += at(k + i, k) * rhs[k + i];
        tmp += rhs[k];
        rhs[k] -= hc[k] * tmp;
        for (int i = 1; i < n; ++i) rhs[k + i] -= hc[k] * at(k + i, k) * tmp;
    }
    for (int i = cols - 1; i >= 0; --i) {
        rhs[i] /= at(i, i);
        for (int s = 0; s < i; ++s) rhs[s] -= rhs[i] * at(s, i);
    }
    for (int j = 0; j < cols; ++j) x[j] = rhs[j];
}

// ---- GPU_EQUIV LM (PFREF_LM_NORMAL_EQ): the device's solve, restated step for step -----------
// pfilter-noetic_amd/csrc/pf_odom.hip k_lm_solve / lm_accept / lm_try_step / lm_next_step. The
// same Ceres 1.14 trust-region loop as solve_lm below, on the 6x6 normal equations (Cholesky) with
// the device's arithmetic order, so that the GPU and this mode agree to the bit over whole
// sequences: every evaluation reduces (cost, g, upper J^T J) over the residuals in the device's
// fixed tree, the Jacobi scaling multiplies H instead of J, and the SE(3) update is se3_plus_half.
constexpr int kDevBlocks = 32;        // pf_odom.hip PF_LM_BLOCKS
constexpr int kDevChunk = 256;        // rows per block pass (threads per block)
constexpr int kDevRows = 29;          // rows per reduction thread: 9 threads per product
constexpr int kDevProducts = 28;      // cost, g[6], upper J^T J (21, row by row)
constexpr int kDevEvals = 5;          // 1 + max_num_iterations

struct DevLm {
    double x[7], cand[7], best[7], scale[6], g[6], H[21], D[6];
    double cost, radius, decrease, x_norm, min_cost, mcc;
    int iteration, invalid, reuse, done, phase;
};
struct DevStep {
    double y[6], D[6], mcc;
    bool ok;
};
inline int hup(int i, int j) {        // packed upper triangle, row by row
    if (i > j) std::swap(i, j);
    return i * 6 - (i * (i - 1)) / 2 + (j - i);
}
inline int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// One evaluation at x. The device's tree: residual q (its query index) is row q % 256 of chunk
// q / 256, chunk n belongs to block n % 32; thread (k, p) of a block sums product k over rows
// 29 p .. 29 p + 28 of each of its chunks, chunk after chunk; the block adds its 9 thread sums in p
// order and the total adds the 32 block sums in block order. Queries without a kept residual (and
// residuals that are not finite) are zero rows there, which leave every partial unchanged, so only
// the kept residuals are visited, in increasing q as the device takes them.
thread_local __float128 g_totq[28];   // PFREF_LM_QUAD: the evaluation's products summed in binary128
thread_local __float128 g_Hq[21], g_gq[6];
void dev_evaluate(const std::vector<Residual>& res, const double* x, double tot[30]) {
    static thread_local std::vector<double> part;
    part.assign((size_t)kDevBlocks * kDevProducts * 9, 0.0);
    for (int k = 0; k < 28; ++k) g_totq[k] = 0;
    int bad_r = 0, bad_j = 0;
    for (const Residual& rs : res) {
        double J[7];
        double r = rs.edge ? edge_eval(x, rs.cur, rs.a, rs.b, rs.w, J) : surf_eval(x, rs.cur, rs.a, rs.d, rs.w, J);
        bool jbad = false;
        for (int k = 0; k < 6; ++k) jbad |= !std::isfinite(J[k]);
        if (!std::isfinite(r)) {
            ++bad_r;
            continue;
        }
        if (jbad) ++bad_j;
        const double s = r * r;                                  // HuberLoss(0.1) + Corrector
        double rho0, rho1;
        if (s > kHuberB) {
            const double rr = std::sqrt(s);
            rho0 = 2.0 * kHuberA * rr - kHuberB;
            rho1 = std::max(std::numeric_limits<double>::min(), kHuberA / rr);
        } else {
            rho0 = s;
            rho1 = 1.0;
        }
        const double hc = 0.5 * rho0;
        const double sr = std::sqrt(rho1);
        r *= sr;
        for (int k = 0; k < 6; ++k) J[k] *= sr;
        const int blk = (rs.q / kDevChunk) % kDevBlocks, p = (rs.q % kDevChunk) / kDevRows;
        double* P = &part[(size_t)blk * kDevProducts * 9 + p];
        P[0] += hc * 1.0;
        for (int k = 0; k < 6; ++k) P[9 * (1 + k)] += J[k] * r;
        int h = 7;
        for (int i = 0; i < 6; ++i)
            for (int j = i; j < 6; ++j, ++h) P[9 * h] += J[i] * J[j];
        if (g_quad) {
            g_totq[0] += (__float128)hc;
            for (int k = 0; k < 6; ++k) g_totq[1 + k] += (__float128)J[k] * (__float128)r;
            int hq = 7;
            for (int i = 0; i < 6; ++i)
                for (int j = i; j < 6; ++j, ++hq) g_totq[hq] += (__float128)J[i] * (__float128)J[j];
        }
    }
    for (int k = 0; k < kDevProducts; ++k) {
        double v = 0.0;
        for (int b = 0; b < kDevBlocks; ++b) {
            const double* P = &part[((size_t)b * kDevProducts + k) * 9];
            double vb = P[0];
            for (int p = 1; p < 9; ++p) vb += P[p];
            v += vb;
        }
        tot[k] = v;
    }
    tot[28] = (double)bad_r;
    tot[29] = (double)bad_j;
}

DevStep dev_try_step(const DevLm& lm) {                       // lm_try_step
    DevStep r;
    for (int j = 0; j < 6; ++j)
        r.D[j] = lm.reuse ? lm.D[j] : std::fmin(std::fmax(lm.scale[j] * lm.H[hup(j, j)] * lm.scale[j], 1e-6), 1e32);
    if (g_quad) {                                            // the same step in binary128 (experiment)
        typedef __float128 Q;
        Q A[21], L[21], d[6], y[6];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j <= i; ++j) A[tri(i, j)] = (Q)lm.scale[i] * g_Hq[hup(i, j)] * (Q)lm.scale[j];
        for (int j = 0; j < 6; ++j) A[tri(j, j)] += (Q)r.D[j] / (Q)lm.radius;
        bool ok = true;
        for (int i = 0; i < 6; ++i) {
            for (int j = 0; j < i; ++j) {
                Q s2 = A[tri(i, j)];
                for (int k = 0; k < j; ++k) s2 -= L[tri(i, k)] * d[k] * L[tri(j, k)];
                L[tri(i, j)] = s2 / d[j];
            }
            Q dd = A[tri(i, i)];
            for (int k = 0; k < i; ++k) dd -= L[tri(i, k)] * L[tri(i, k)] * d[k];
            ok = ok && dd > 0;
            d[i] = dd;
        }
        for (int i = 0; i < 6; ++i) {
            Q s2 = (Q)lm.scale[i] * g_gq[i];
            for (int k = 0; k < i; ++k) s2 -= L[tri(i, k)] * y[k];
            y[i] = s2;
        }
        for (int i = 5; i >= 0; --i) {
            Q s2 = y[i] / d[i];
            for (int k = i + 1; k < 6; ++k) s2 -= L[tri(k, i)] * y[k];
            y[i] = s2;
        }
        for (int j = 0; j < 6; ++j) { r.y[j] = (double)y[j]; ok = ok && std::isfinite(r.y[j]); }
        r.mcc = 0.0;
        if (ok) {
            Q sg = 0, sHs = 0;
            for (int i = 0; i < 6; ++i) {
                sg -= y[i] * (Q)lm.scale[i] * g_gq[i];
                Q hi = 0;
                for (int j = 0; j < 6; ++j) hi -= (Q)lm.scale[i] * g_Hq[hup(i, j)] * (Q)lm.scale[j] * y[j];
                sHs -= y[i] * hi;
            }
            r.mcc = (double)(-(sg + sHs / 2));
        }
        r.ok = ok && r.mcc > 0.0;
        return r;
    }
    // Hs + D / radius (D times the reciprocal radius), LDL^T with reciprocal pivots: the device's
    // operation order (W_ij = L_ij d_j accumulated first, L_ij = W_ij / d_j as a product) and its
    // fused multiply-adds (std::fma: one rounding, as v_fma_f64)
    double A[21];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j <= i; ++j) A[tri(i, j)] = lm.scale[i] * lm.H[hup(i, j)] * lm.scale[j];
    const double ir = 1.0 / lm.radius;
    for (int j = 0; j < 6; ++j) A[tri(j, j)] += r.D[j] * ir;
    double W[21], inv[6];
    bool ok = true;
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < i; ++j) {
            double s = A[tri(i, j)];
            for (int k = 0; k < j; ++k) s = std::fma(-W[tri(i, k)], A[tri(j, k)], s);
            W[tri(i, j)] = s;
            A[tri(i, j)] = s * inv[j];
        }
        double d = A[tri(i, i)];
        for (int k = 0; k < i; ++k) d = std::fma(-W[tri(i, k)], A[tri(i, k)], d);
        ok = ok && (d > 0.0);
        inv[i] = 1.0 / d;
    }
    for (int i = 0; i < 6; ++i) {                               // L z = scale .* g
        double s = lm.scale[i] * lm.g[i];
        for (int k = 0; k < i; ++k) s = std::fma(-A[tri(i, k)], r.y[k], s);
        r.y[i] = s;
    }
    for (int i = 5; i >= 0; --i) {                              // L^T y = D^-1 z
        double s = r.y[i] * inv[i];
        for (int k = i + 1; k < 6; ++k) s = std::fma(-A[tri(k, i)], r.y[k], s);
        r.y[i] = s;
    }
    for (int j = 0; j < 6; ++j) ok = ok && std::isfinite(r.y[j]);
    r.mcc = 0.0;
    if (ok) {
        double sg = 0.0, sHs = 0.0;
        for (int i = 0; i < 6; ++i) {
            sg = std::fma(-r.y[i], lm.scale[i] * lm.g[i], sg);
            double hi = 0.0;
            for (int j = 0; j < 6; ++j) hi = std::fma(lm.scale[i] * lm.H[hup(i, j)] * lm.scale[j], -r.y[j], hi);
            sHs = std::fma(-r.y[i], hi, sHs);
        }
        r.mcc = -(sg + 0.5 * sHs);
    }
    r.ok = ok && (r.mcc > 0.0);
    return r;
}

void dev_next_step(DevLm& lm, DevStep st, const double* cand_first) {   // lm_next_step
    const int kMaxIter = 4;
    for (bool first = true;; first = false) {
        lm.iteration++;
        if (!first) st = dev_try_step(lm);
        if (!lm.reuse)
            for (int j = 0; j < 6; ++j) lm.D[j] = st.D[j];
        lm.reuse = 1;
        if (!st.ok) {
            if (++lm.invalid >= 5) { lm.done = 1; return; }
            lm.radius = lm.radius / lm.decrease;
            lm.decrease *= 2.0;
            if (lm.iteration >= kMaxIter || lm.radius <= 1e-32) { lm.done = 1; return; }
            continue;
        }
        lm.invalid = 0;
        if (first) {
            for (int k = 0; k < 7; ++k) lm.cand[k] = cand_first[k];
        } else {
            double delta[6];
            for (int j = 0; j < 6; ++j) delta[j] = -st.y[j] * lm.scale[j];
            if (g_dev_libm) se3_plus(lm.x, delta, lm.cand);
            else se3_plus_half(lm.x, delta, lm.cand);
        }
        lm.mcc = st.mcc;
        lm.phase = 1;
        return;
    }
}

void dev_accept(DevLm& lm, const double* tot) {                     // lm_accept
    const double cost_c = tot[0];
    const bool bad_r = tot[28] > 0.0, bad_j = tot[29] > 0.0;
    const int kMaxIter = 4;
    bool step_ok = false;
    if (lm.phase == 0) {
        if (bad_r || bad_j) { lm.done = 1; return; }
        lm.cost = cost_c;
        for (int k = 0; k < 6; ++k) lm.g[k] = tot[1 + k];
        for (int k = 0; k < 21; ++k) lm.H[k] = tot[7 + k];
        for (int k = 0; k < 6; ++k) g_gq[k] = g_totq[1 + k];
        for (int k = 0; k < 21; ++k) g_Hq[k] = g_totq[7 + k];
        for (int i = 0; i < 6; ++i) lm.scale[i] = 1.0 / (1.0 + std::sqrt(lm.H[hup(i, i)]));
        lm.min_cost = lm.cost;
        for (int k = 0; k < 7; ++k) lm.best[k] = lm.x[k];
        step_ok = true;
    } else {
        const double cand_cost = bad_r ? DBL_MAX : cost_c;
        double sn = 0.0;
        for (int j = 0; j < 7; ++j) sn += (lm.x[j] - lm.cand[j]) * (lm.x[j] - lm.cand[j]);
        sn = std::sqrt(sn);
        if (sn <= 1e-8 * (lm.x_norm + 1e-8)) { lm.done = 1; return; }
        if (std::fabs(lm.cost - cand_cost) <= 1e-6 * lm.cost) { lm.done = 1; return; }
        const double rel = (lm.cost - cand_cost) / lm.mcc;
        if (rel > 1e-3) {
            double xn = 0;
            for (int j = 0; j < 7; ++j) { lm.x[j] = lm.cand[j]; xn += lm.x[j] * lm.x[j]; }
            lm.x_norm = std::sqrt(xn);
            if (bad_j) { lm.done = 1; return; }
            lm.cost = cand_cost;
            for (int k = 0; k < 6; ++k) lm.g[k] = tot[1 + k];
            for (int k = 0; k < 21; ++k) lm.H[k] = tot[7 + k];
            for (int k = 0; k < 6; ++k) g_gq[k] = g_totq[1 + k];
            for (int k = 0; k < 21; ++k) g_Hq[k] = g_totq[7 + k];
            const double r3 = 2.0 * rel - 1.0;
            const double f = 1.0 - r3 * r3 * r3;
            lm.radius = lm.radius / std::fmax(1.0 / 3.0, f);
            lm.radius = std::fmin(1e16, lm.radius);
            lm.decrease = 2.0;
            lm.reuse = 0;
            step_ok = true;
            if (lm.cost < lm.min_cost) {
                lm.min_cost = lm.cost;
                for (int k = 0; k < 7; ++k) lm.best[k] = lm.x[k];
            }
        } else {
            lm.radius = lm.radius / lm.decrease;
            lm.decrease *= 2.0;
            lm.reuse = 1;
        }
        if (lm.iteration >= kMaxIter) { lm.done = 1; return; }
    }
    const DevStep st = dev_try_step(lm);
    double ng[6], gx[7], delta[6], cand[7];
    for (int j = 0; j < 6; ++j) { ng[j] = -lm.g[j]; delta[j] = -st.y[j] * lm.scale[j]; }
    if (g_dev_libm) {
        se3_plus(lm.x, ng, gx);
        se3_plus(lm.x, delta, cand);
    } else {
        se3_plus_half(lm.x, ng, gx);                             // gradient max-norm check
        se3_plus_half(lm.x, delta, cand);                        // the first attempt's candidate
    }
    double gm = 0.0;
    for (int j = 0; j < 7; ++j) gm = std::fmax(gm, std::fabs(lm.x[j] - gx[j]));
    if (step_ok && gm <= 1e-10) lm.done = 1;
    else if (lm.phase != 0 && lm.radius <= 1e-32) lm.done = 1;
    else dev_next_step(lm, st, cand);
}

// Returns the LM iterations; params becomes the best point (unchanged without residuals).
int solve_lm_dev(double* params, const std::vector<Residual>& res) {
    if (res.empty()) return 0;
    DevLm lm{};
    double xn = 0;
    for (int k = 0; k < 7; ++k) {
        lm.x[k] = lm.cand[k] = lm.best[k] = params[k];
        xn += lm.x[k] * lm.x[k];
    }
    lm.x_norm = std::sqrt(xn);
    lm.radius = 1e4;
    lm.decrease = 2.0;
    for (int ev = 0; ev < kDevEvals; ++ev) {
        if (lm.done) break;
        double tot[30];
        dev_evaluate(res, lm.cand, tot);
        dev_accept(lm, tot);
        if (ev == kDevEvals - 1) lm.done = 1;
    }
    std::copy(lm.best, lm.best + 7, params);
    return lm.iteration;
}

double grad_max_norm(const double* x, const double* g) {
    double ng[6], xp[7];
    for (int j = 0; j < 6; ++j) ng[j] = -g[j];
    se3_plus(x, ng, xp);
    double m = 0.0;
    for (int j = 0; j < 7; ++j) m = std::max(m, std::fabs(x[j] - xp[j]));
    return m;
}
}  // namespace

// Returns the number of LM iterations performed. params is updated with the best point.
int solve_lm(double* params, const std::vector<Residual>& res, bool normal_eq) {
    if (normal_eq) return solve_lm_dev(params, res);
    const int m = (int)res.size();
    if (m == 0) return 0;  // no residual blocks: parameter block removed, nothing to do
    const int kMaxIter = 4;
    double x[7];
    std::copy(params, params + 7, x);
    double x_norm = 0.0;
    for (int j = 0; j < 7; ++j) x_norm += x[j] * x[j];
    x_norm = std::sqrt(x_norm);
    double radius = 1e4, decrease_factor = 2.0;
    bool reuse_diag = false;
    int invalid = 0;
    std::vector<double> r(m), J(6 * (size_t)m);
    double cost;
    if (!evaluate(res, x, cost, &r, &J)) return 0;                // FAILURE, params unchanged
    double scale[6], D[6], g[6];
    auto grad = [&]() {
        for (int j = 0; j < 6; ++j) g[j] = 0.0;
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < 6; ++j) g[j] += J[6 * (size_t)i + j] * r[i];
    };
    for (int j = 0; j < 6; ++j) {                                  // Jacobi scaling, iteration 0
        double s = 0.0;
        for (int i = 0; i < m; ++i) s += J[6 * (size_t)i + j] * J[6 * (size_t)i + j];
        scale[j] = 1.0 / (1.0 + std::sqrt(s));
    }
    grad();
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < 6; ++j) J[6 * (size_t)i + j] *= scale[j];
    double gmax = grad_max_norm(x, g);
    double min_cost = cost;
    std::copy(x, x + 7, params);
    int iteration = 0;
    if (gmax <= 1e-10) return iteration;
    std::vector<double> mr(m), A, rhs;
    while (true) {
        ++iteration;
        bool step_ok = false;
        if (!reuse_diag) {
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int i = 0; i < m; ++i) s += J[6 * (size_t)i + j] * J[6 * (size_t)i + j];
                D[j] = std::min(std::max(s, 1e-6), 1e32);
            }
        }
        double lm_diag[6], y[6], step[6];
        for (int j = 0; j < 6; ++j) lm_diag[j] = std::sqrt(D[j] / radius);
        bool solved = true;
        {
            const int rows = m + 6;
            A.assign((size_t)rows * 6, 0.0);
            rhs.assign(rows, 0.0);
            for (int j = 0; j < 6; ++j) {
                for (int i = 0; i < m; ++i) A[(size_t)j * rows + i] = J[6 * (size_t)i + j];
                A[(size_t)j * rows + m + j] = lm_diag[j];
            }
            for (int i = 0; i < m; ++i) rhs[i] = r[i];
            householder_solve(A, rows, 6, rhs, y);
        }
        for (int j = 0; j < 6; ++j) if (!std::isfinite(y[j])) solved = false;
        reuse_diag = true;
        double mcc = 0.0;
        if (solved) {
            for (int j = 0; j < 6; ++j) step[j] = -y[j];
            for (int i = 0; i < m; ++i) {
                double s = 0.0;
                for (int j = 0; j < 6; ++j) s += J[6 * (size_t)i + j] * step[j];
                mr[i] = s;
            }
            for (int i = 0; i < m; ++i) mcc += mr[i] * (r[i] + mr[i] / 2.0);
            mcc = -mcc;
        }
        if (!solved || !(mcc > 0.0)) {                            // invalid step
            if (++invalid >= 5) return iteration;                  // FAILURE (best point kept)
            radius = radius / decrease_factor;
            decrease_factor *= 2.0;
        } else {
            invalid = 0;
            double delta[6], cand[7];
            for (int j = 0; j < 6; ++j) delta[j] = step[j] * scale[j];
            se3_plus(x, delta, cand);
            double cand_cost;
            if (!evaluate(res, cand, cand_cost, nullptr, nullptr)) cand_cost = DBL_MAX;
            double sn = 0.0;
            for (int j = 0; j < 7; ++j) sn += (x[j] - cand[j]) * (x[j] - cand[j]);
            sn = std::sqrt(sn);
            if (sn <= 1e-8 * (x_norm + 1e-8)) return iteration;    // parameter tolerance
            double cost_change = cost - cand_cost;
            if (std::fabs(cost_change) <= 1e-6 * cost) return iteration;  // function tolerance
            double rel = (cost - cand_cost) / mcc;
            if (rel > 1e-3) {                                      // successful step
                std::copy(cand, cand + 7, x);
                x_norm = 0.0;
                for (int j = 0; j < 7; ++j) x_norm += x[j] * x[j];
                x_norm = std::sqrt(x_norm);
                if (!evaluate(res, x, cost, &r, &J)) return iteration;  // FAILURE
                grad();
                for (int i = 0; i < m; ++i)
                    for (int j = 0; j < 6; ++j) J[6 * (size_t)i + j] *= scale[j];
                gmax = grad_max_norm(x, g);
                trig_dump(-1e300);                                  // marks the next value: a cube base
                trig_dump(2.0 * rel - 1.0);
                radius = radius / std::max(1.0 / 3.0, 1.0 - lcube(2.0 * rel - 1.0));
                radius = std::min(1e16, radius);
                decrease_factor = 2.0;
                reuse_diag = false;
                step_ok = true;
                if (cost < min_cost) { min_cost = cost; std::copy(x, x + 7, params); }
            } else {
                radius = radius / decrease_factor;
                decrease_factor *= 2.0;
                reuse_diag = true;
            }
        }
        if (iteration >= kMaxIter) return iteration;
        if (step_ok && gmax <= 1e-10) return iteration;
        if (radius <= 1e-32) return iteration;
    }
}

// ------------------------------------------------------------------------------------------
// Odom_ES_EstimationClass (src/odomEstimationClass.cpp:182-647)
// ------------------------------------------------------------------------------------------
struct Odom {
    pfref_lidar lidar;
    int opts;
    float map_resolution;
    // map classes: ES = {corner (line), surf (plane)}; BPF = {beam (line), pillar (line), facade (plane)}
    int nc = 2;
    bool plane[3] = {false, true, true};
    float leaf_vg[3];                   // downSizeFilter leaf sizes (double -> float)
    float leaf_rg[3];                   // rgbds leaves (float map_resolution, times 2 for planes)
    int k_new_edge, k_new_surf;
    float theta_p_edge, theta_p_surf;
    int theta_max_edge, theta_max_surf;
    double weightType;
    double params[7] = {0, 0, 0, 1, 0, 0, 0};
    Iso odom, last_odom;
    int optimization_count;
    std::vector<PtC> maps[3];           // laserCloudCornerMap / SurfMap, or Beam / Pillar / FacadeMap
    KdTree trees[3];
    pfref_stats stats{};

    Quat q() const { return {params[0], params[1], params[2], params[3]}; }
    V3 t() const { return {params[4], params[5], params[6]}; }

    // pointAssociateToMap (:162-174)
    PtC associate(const PtC& pi) const {
        V3 pw = add(qrot(q(), V3{(double)pi.x, (double)pi.y, (double)pi.z}), t());
        PtC po;
        po.x = (float)pw.x; po.y = (float)pw.y; po.z = (float)pw.z;
        po.r = pi.r; po.g = pi.g; po.b = pi.b;
        return po;
    }

    void knn(int c, const PtC& p, int* ind, float* d2) const {
        const float qq[3] = {p.x, p.y, p.z};
        if (opts & PFREF_KNN_BRUTE) knn_brute(maps[c], qq, 5, ind, d2);
        else trees[c].knn(qq, 5, ind, d2);
    }
    int k_new(int c) const { return plane[c] ? k_new_surf : k_new_edge; }
    float theta_p(int c) const { return plane[c] ? theta_p_surf : theta_p_edge; }
    int theta_max(int c) const { return plane[c] ? theta_max_surf : theta_max_edge; }
};

namespace {
// observeMean (:136-160) / pointSparsityMean (include/odomEstimationClass.h:111-126)
void observe_mean(std::vector<double>& v) {
    if (v.empty()) return;
    double mn = *std::min_element(v.begin(), v.end());
    double mx = *std::max_element(v.begin(), v.end());
    double length = mx - mn;
    if (length == 0) return;
    for (double& e : v) {
        e = (e - mn) / length;
        e -= 1.0;
        e = std::fabs(e);   // abs() binds to the double overload (<math.h>), A.11
        e *= 2.0;
        e = std::max(0.1, e);
    }
}
void sparsity_mean(std::vector<double>& v) {
    if (v.empty()) return;
    double mn = *std::min_element(v.begin(), v.end());
    double mx = *std::max_element(v.begin(), v.end());
    double length = mx - mn;
    if (length == 0) return;
    for (double& e : v) {
        e = (e - mn) / length;
        e -= 1.0;
        e = std::fabs(e);
        e *= 2.0;
    }
}

// observe / round from the 5 neighbours, increments, skip test (:332-356 / :480-504)
// returns true when the query is kept
bool pindex(std::vector<PtC>& map, const int* ind, int k_new, float theta_p, int theta_max, float& observe,
            float& round) {
    observe = (map[ind[0]].g + map[ind[1]].g + map[ind[2]].g + map[ind[3]].g + map[ind[4]].g) / 5.0 + 1;
    round = (map[ind[0]].r + map[ind[1]].r + map[ind[2]].r + map[ind[3]].r + map[ind[4]].r) / 5.0;
    for (int j = 0; j < 5; j++) map[ind[j]].g = (uint8_t)std::min(255, map[ind[j]].g + 1);
    if (observe / round > 5) observe = 255;
    if (observe < round * theta_p && round > k_new && observe < theta_max) return false;
    return true;
}

// float sum of distances to the neighbour centroid / 5 (:367-385)
double sparsity(const std::vector<PtC>& map, const int* ind) {
    float sum = 0;
    V3 c{0, 0, 0};
    V3 p[5];
    for (int j = 0; j < 5; j++) {
        p[j] = V3{(double)map[ind[j]].x, (double)map[ind[j]].y, (double)map[ind[j]].z};
        c = add(c, p[j]);
    }
    c = V3{c.x / 5, c.y / 5, c.z / 5};
    for (int j = 0; j < 5; j++) sum += norm(sub(c, p[j]));
    sum /= 5.0;
    return (double)sum;
}
}  // namespace

// addEdgeCostFactor (:284-432); Odom_BPF addBeamCostFactor / addPillarCostFactor (:751-1010) are
// the same function of their own map with the edge thresholds
static void add_line_factors(Odom& o, int c, std::vector<PtC>& cloud, int qbase, std::vector<Residual>& out) {
    struct Info { V3 cur, a, b; float observe, round; int q; };
    std::vector<Info> valid;
    std::vector<double> spars, obs;
    std::vector<PtC>& map = o.maps[c];
    int64_t n_valid = 0;
    for (size_t i = 0; i < cloud.size(); i++) {
        PtC pt = o.associate(cloud[i]);
        int ind[5]; float d2[5];
        o.knn(c, pt, ind, d2);
        if (!(d2[4] < 1.0)) continue;
        V3 near[5];
        V3 center{0, 0, 0};
        for (int j = 0; j < 5; j++) {
            near[j] = V3{(double)map[ind[j]].x, (double)map[ind[j]].y, (double)map[ind[j]].z};
            center = add(center, near[j]);
        }
        center = V3{center.x / 5.0, center.y / 5.0, center.z / 5.0};
        double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        for (int j = 0; j < 5; j++) {
            V3 t = sub(near[j], center);
            const double tv[3] = {t.x, t.y, t.z};
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) cov[a][b] = cov[a][b] + tv[a] * tv[b];
        }
        double ev[3], V[3][3];
        eigen_sym3(cov, ev, V);
        V3 dir{V[0][2], V[1][2], V[2][2]};
        V3 cur{(double)cloud[i].x, (double)cloud[i].y, (double)cloud[i].z};
        if (ev[2] > 3 * ev[1]) {
            ++n_valid;
            V3 a{0.1 * dir.x + center.x, 0.1 * dir.y + center.y, 0.1 * dir.z + center.z};
            V3 b{-0.1 * dir.x + center.x, -0.1 * dir.y + center.y, -0.1 * dir.z + center.z};
            float observe, round;
            if (!pindex(map, ind, o.k_new(c), o.theta_p(c), o.theta_max(c), observe, round)) continue;
            cloud[i].r = (uint8_t)std::min(255, int(round));
            cloud[i].g = (uint8_t)std::min(255, int(observe));
            valid.push_back({cur, a, b, observe, round, qbase + (int)i});
            spars.push_back(sparsity(map, ind));
        }
    }
    const double wt = o.weightType;
    if (wt == 1 || wt == 12) {
        for (const Info& v : valid) obs.push_back(v.observe);
        observe_mean(obs);
    }
    if (wt == 2 || wt == 12) sparsity_mean(spars);
    for (size_t i = 0; i < valid.size(); i++) {
        Residual r;
        r.edge = true; r.cur = valid[i].cur; r.a = valid[i].a; r.b = valid[i].b; r.d = 0; r.q = valid[i].q;
        if (wt == 0) r.w = 0;
        else if (wt == 1) r.w = obs[i];
        else if (wt == 2) r.w = spars[i];
        else r.w = (spars[i] + obs[i]) / 2;
        out.push_back(r);
    }
    o.stats.n_res[c] = (int64_t)valid.size();
    o.stats.n_valid[c] = n_valid;
}

// addSurfCostFactor (:434-578); Odom_BPF addFacadeCostFactor (:1012-1193) with the surf thresholds
static void add_plane_factors(Odom& o, int c, std::vector<PtC>& cloud, int qbase, std::vector<Residual>& out) {
    struct Info { V3 cur, n; float d, observe, round; int q; };
    std::vector<Info> valid;
    std::vector<double> spars, obs;
    std::vector<PtC>& map = o.maps[c];
    int64_t n_valid = 0;
    for (size_t i = 0; i < cloud.size(); i++) {
        PtC pt = o.associate(cloud[i]);
        int ind[5]; float d2[5];
        o.knn(c, pt, ind, d2);
        if (!(d2[4] < 1.0)) continue;
        double A[5][3];
        for (int j = 0; j < 5; j++) {
            A[j][0] = map[ind[j]].x; A[j][1] = map[ind[j]].y; A[j][2] = map[ind[j]].z;
        }
        V3 n = plane_fit5(A);
        double negative_OA_dot_norm = 1 / norm(n);
        double z = sqnorm(n);
        if (z > 0.0) { double s = std::sqrt(z); n = V3{n.x / s, n.y / s, n.z / s}; }
        bool planeValid = true;
        for (int j = 0; j < 5; j++) {
            if (std::fabs(n.x * map[ind[j]].x + n.y * map[ind[j]].y + n.z * map[ind[j]].z +
                          negative_OA_dot_norm) > 0.2) {
                planeValid = false;
                break;
            }
        }
        V3 cur{(double)cloud[i].x, (double)cloud[i].y, (double)cloud[i].z};
        if (planeValid) {
            ++n_valid;
            float observe, round;
            if (!pindex(map, ind, o.k_new(c), o.theta_p(c), o.theta_max(c), observe, round)) continue;
            cloud[i].r = (uint8_t)std::min(255, int(round));
            cloud[i].g = (uint8_t)std::min(255, int(observe));
            valid.push_back({cur, n, (float)negative_OA_dot_norm, observe, round, qbase + (int)i});
            spars.push_back(sparsity(map, ind));
        }
    }
    const double wt = o.weightType;
    if (wt == 1 || wt == 12) {
        for (const Info& v : valid) obs.push_back(v.observe);
        observe_mean(obs);
    }
    if (wt == 2 || wt == 12) sparsity_mean(spars);
    for (size_t i = 0; i < valid.size(); i++) {
        Residual r;
        r.edge = false; r.cur = valid[i].cur; r.a = valid[i].n; r.b = V3{0, 0, 0}; r.q = valid[i].q;
        r.d = (double)valid[i].d;       // float member of surfInfo, reloaded into a float (A.7)
        if (wt == 0) r.w = 0;
        else if (wt == 1) r.w = obs[i];
        else if (wt == 2) r.w = spars[i];
        else r.w = (obs[i] + spars[i]) / 2;
        out.push_back(r);
    }
    o.stats.n_res[c] = (int64_t)valid.size();
    o.stats.n_valid[c] = n_valid;
}

// extractstablepoint (:7-25)
static void extract_stable(std::vector<PtC>& m, int k_new, float theta_p, int theta_max) {
    std::vector<PtC> keep;
    keep.reserve(m.size());
    for (const PtC& p : m) {
        if (p.g < p.r * theta_p && p.r > k_new && p.g < theta_max + 1) continue;
        keep.push_back(p);
    }
    m.swap(keep);
}

// addPointsToMap (:589-647; BPF :1197-1290): append every class, CropBox +-100 m around odom.t,
// rgbds with the class leaf, extractstablepoint with the class thresholds, ageing. The classes are
// independent maps, so the reference's order across them (surf before corner, facade first) is moot.
static void add_points_to_map(Odom& o, const std::vector<PtC>* ds) {
    const bool stable = (o.opts & PFREF_VG_STABLE) != 0;
    for (int c = 0; c < o.nc; ++c)
        for (const PtC& p : ds[c]) o.maps[c].push_back(o.associate(p));
    const double tx = o.odom.t.x, ty = o.odom.t.y, tz = o.odom.t.z;
    const float mn[3] = {(float)(tx - 100), (float)(ty - 100), (float)(tz - 100)};
    const float mx[3] = {(float)(tx + 100), (float)(ty + 100), (float)(tz + 100)};
    auto crop = [&](const std::vector<PtC>& in, std::vector<PtC>& out) {  // CropBox (B.2)
        out.clear();
        for (const PtC& p : in) {
            if ((p.x < mn[0] || p.y < mn[1] || p.z < mn[2]) || (p.x > mx[0] || p.y > mx[1] || p.z > mx[2])) continue;
            out.push_back(p);
        }
    };
    for (int c = 0; c < o.nc; ++c) {
        std::vector<PtC> tmp;
        crop(o.maps[c], tmp);
        rgbds(tmp, o.leaf_rg[c], stable, o.maps[c]);
        extract_stable(o.maps[c], o.k_new(c), o.theta_p(c), o.theta_max(c));
        for (PtC& p : o.maps[c]) p.r = p.r > 250 ? 255 : (uint8_t)(p.r + 2);
    }
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void legacy_stats(Odom& o) {       // ES field names: class 0 = edge, class 1 = surf
    pfref_stats& st = o.stats;
    st.n_edge_in = st.n_in[0]; st.n_surf_in = st.n_in[1];
    st.n_edge_ds = st.n_ds[0]; st.n_surf_ds = st.n_ds[1];
    st.n_edge_map = st.n_map[0]; st.n_surf_map = st.n_map[1];
    st.n_edge_res = st.n_res[0]; st.n_surf_res = st.n_res[1];
    st.n_edge_valid = st.n_valid[0]; st.n_surf_valid = st.n_valid[1];
}

// updatePointsToMap: ES :229-282, BPF :702-749 (the same sequence over 2 or 3 map classes)
int odom_update(Odom& o, const std::vector<PtC>* in) {
    pfref_stats& st = o.stats;
    st = pfref_stats{};
    for (int c = 0; c < o.nc; ++c) st.n_in[c] = (int64_t)in[c].size();
    if (o.optimization_count > 2) o.optimization_count--;               // :232-233
    Iso pred = iso_mul(o.odom, iso_mul(iso_inv(o.last_odom), o.odom)); // :235-237
    o.last_odom = o.odom;
    o.odom = pred;
    Quat q = m2q(rotation_polar(o.odom.R));                             // :239 (Eigen 3.3 rotation())
    o.params[0] = q.x; o.params[1] = q.y; o.params[2] = q.z; o.params[3] = q.w;
    o.params[4] = o.odom.t.x; o.params[5] = o.odom.t.y; o.params[6] = o.odom.t.z;
    const bool stable = (o.opts & PFREF_VG_STABLE) != 0;
    double t0 = now_s();
    std::vector<PtC> ds[3];
    for (int c = 0; c < o.nc; ++c) {                                    // :242-245 / :714-719
        voxel_grid(in[c], o.leaf_vg[c], stable, ds[c]);
        st.n_ds[c] = (int64_t)ds[c].size();
    }
    double t1 = now_s();
    st.t_downsample = t1 - t0;
    bool big_enough = true;                                             // :247 / :721
    for (int c = 0; c < o.nc; ++c) big_enough = big_enough && o.maps[c].size() > (o.plane[c] ? 50u : 10u);
    if (big_enough) {
        if (!(o.opts & PFREF_KNN_BRUTE))
            for (int c = 0; c < o.nc; ++c) o.trees[c].build(o.maps[c]);
        double t2 = now_s();
        st.t_tree = t2 - t1;
        st.outer_iterations = o.optimization_count;
        for (int it = 0; it < o.optimization_count; it++) {           // :252-272 / :727-747
            double ta = now_s();
            std::vector<Residual> res;
            int qbase = 0;
            for (int c = 0; c < o.nc; ++c) {
                if (o.plane[c]) add_plane_factors(o, c, ds[c], qbase, res);
                else add_line_factors(o, c, ds[c], qbase, res);
                qbase += (int)ds[c].size();
            }
            double tb = now_s();
            g_ld_trig = (o.opts & PFREF_LD_TRIG) != 0;
            g_qr_rev = (o.opts & PFREF_QR_REVSUM) != 0;
            g_quad = (o.opts & PFREF_LM_QUAD) != 0;
            g_cost_rev = (o.opts & PFREF_COST_REVSUM) != 0;
            g_dev_libm = (o.opts & PFREF_DEV_LIBM) != 0;
            g_dev_half = (o.opts & PFREF_DEV_HALFANGLE) != 0;
            st.lm_iterations += solve_lm(o.params, res, (o.opts & PFREF_LM_NORMAL_EQ) != 0);
            g_ld_trig = g_qr_rev = g_quad = g_cost_rev = g_dev_libm = g_dev_half = false;
            double tc = now_s();
            st.t_assoc += tb - ta;
            st.t_solve += tc - tb;
        }
    } else {
        std::printf("not enough points in map to associate, map error");
        st.map_too_small = 1;
    }
    double t3 = now_s();
    o.odom = iso_identity();                                             // :278-280
    o.odom.R = q2m(o.q());
    o.odom.t = o.t();
    add_points_to_map(o, ds);                                            // :281
    st.t_mapupdate = now_s() - t3;
    for (int c = 0; c < o.nc; ++c) st.n_map[c] = (int64_t)o.maps[c].size();
    legacy_stats(o);
    return 0;
}

}  // namespace pfref

// ==========================================================================================
// C ABI
// ==========================================================================================
using namespace pfref;

struct pfref_odom { Odom o; bool inited = false; };

static std::vector<PtC> to_ptc(const float* xyzi, size_t n) {   // pcl::copyPointCloud XYZI->XYZRGB
    std::vector<PtC> v(n);
    for (size_t i = 0; i < n; ++i) {
        v[i].x = xyzi[4 * i]; v[i].y = xyzi[4 * i + 1]; v[i].z = xyzi[4 * i + 2];
        v[i].r = v[i].g = v[i].b = 0;
    }
    return v;
}

static std::vector<PtC> unpack_rgb(const float* pts, size_t n) {
    std::vector<PtC> v(n);
    for (size_t i = 0; i < n; ++i) {
        uint32_t rgb;
        std::memcpy(&rgb, &pts[4 * i + 3], 4);
        v[i].x = pts[4 * i]; v[i].y = pts[4 * i + 1]; v[i].z = pts[4 * i + 2];
        v[i].r = (rgb >> 16) & 255; v[i].g = (rgb >> 8) & 255; v[i].b = rgb & 255;
    }
    return v;
}
static void pack_rgb(const std::vector<PtC>& v, float* out) {
    for (size_t i = 0; i < v.size(); ++i) {
        uint32_t rgb = ((uint32_t)v[i].r << 16) | ((uint32_t)v[i].g << 8) | v[i].b;
        out[4 * i] = v[i].x; out[4 * i + 1] = v[i].y; out[4 * i + 2] = v[i].z;
        std::memcpy(&out[4 * i + 3], &rgb, 4);
    }
}

extern "C" {

int pfref_feature_extraction(const pfref_lidar* lidar, int opts, const float* xyzi, size_t n, float* edge_out,
                             size_t* n_edge, float* surf_out, size_t* n_surf, size_t cap) {
    std::vector<PtI> e, s;
    feature_extraction(*lidar, opts, reinterpret_cast<const PtI*>(xyzi), n, e, s);
    *n_edge = e.size();
    *n_surf = s.size();
    if (e.size() > cap || s.size() > cap) return -1;
    std::memcpy(edge_out, e.data(), e.size() * sizeof(PtI));
    std::memcpy(surf_out, s.data(), s.size() * sizeof(PtI));
    return 0;
}

int pfref_voxel_grid(const float* pts, size_t n, float leaf, int opts, float* out, size_t* n_out) {
    std::vector<PtC> o;
    voxel_grid(unpack_rgb(pts, n), leaf, (opts & PFREF_VG_STABLE) != 0, o);
    *n_out = o.size();
    pack_rgb(o, out);
    return 0;
}

int pfref_rgbds(const float* pts, size_t n, float leaf, int opts, float* out, size_t* n_out) {
    std::vector<PtC> o;
    rgbds(unpack_rgb(pts, n), leaf, (opts & PFREF_VG_STABLE) != 0, o);
    *n_out = o.size();
    pack_rgb(o, out);
    return 0;
}

int pfref_knn(const float* map, size_t m, const float* queries, size_t q, int k, int opts, int32_t* idx_out,
              float* d2_out) {
    if (k < 1 || k > 8) return -1;
    std::vector<PtC> mp = unpack_rgb(map, m);
    KdTree t;
    if (!(opts & PFREF_KNN_BRUTE)) t.build(mp);
    for (size_t i = 0; i < q; ++i) {
        const float* qq = queries + 4 * i;
        int ind[8]; float d2[8];
        if (opts & PFREF_KNN_BRUTE) knn_brute(mp, qq, k, ind, d2);
        else t.knn(qq, k, ind, d2);
        for (int j = 0; j < k; ++j) { idx_out[i * k + j] = ind[j]; d2_out[i * k + j] = d2[j]; }
    }
    return 0;
}

// Sum over the queries of |C(q)|: the map points in the 3 x 3 x 3 block of 1 m cells (cell =
// floor(p / 1 m)) around each query's cell, the set any exact 5-NN under the d^2 < 1 gate of
// src/odomEstimationClass.cpp:299-300 / :447-451 must inspect (algorithmic bytes).
unsigned long long pfref_knn_cellpop(const float* map, size_t m, const float* queries, size_t q) {
    auto cell = [](const float* p) {
        return std::array<long long, 3>{(long long)std::floor(p[0]), (long long)std::floor(p[1]),
                                        (long long)std::floor(p[2])};
    };
    std::map<std::array<long long, 3>, unsigned long long> count;
    for (size_t i = 0; i < m; ++i) ++count[cell(map + 4 * i)];
    unsigned long long total = 0;
    for (size_t i = 0; i < q; ++i) {
        const auto c = cell(queries + 4 * i);
        for (long long dz = -1; dz <= 1; ++dz)
            for (long long dy = -1; dy <= 1; ++dy)
                for (long long dx = -1; dx <= 1; ++dx) {
                    const auto it = count.find({c[0] + dx, c[1] + dy, c[2] + dz});
                    if (it != count.end()) total += it->second;
                }
    }
    return total;
}

void pfref_eigen_sym3(const double a[6], double evals[3], double evecs[9]) {
    double A[3][3] = {{a[0], a[1], a[2]}, {a[1], a[3], a[4]}, {a[2], a[4], a[5]}};
    double V[3][3];
    eigen_sym3(A, evals, V);
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) evecs[c * 3 + r] = V[r][c];
}

void pfref_plane_fit(const double A[15], double n_out[3]) {
    double M[5][3];
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 3; ++j) M[i][j] = A[i * 3 + j];
    V3 n = plane_fit5(M);
    n_out[0] = n.x; n_out[1] = n.y; n_out[2] = n.z;
}

void pfref_se3_plus(const double x[7], const double delta[6], double out[7]) { se3_plus(x, delta, out); }
void pfref_se3_plus_half(const double x[7], const double delta[6], double out[7]) { se3_plus_half(x, delta, out); }
void pfref_det_sincos(double x, double* s, double* c) { det_sincos(x, s, c); }

void pfref_rotation_polar(const double m[9], double out[9]) {
    M3 a;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) a.m[i][j] = m[3 * i + j];
    const M3 r = rotation_polar(a);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out[3 * i + j] = r.m[i][j];
}

double pfref_edge_eval(const double x[7], const double cur[3], const double a[3], const double b[3], double weight,
                       double J[7]) {
    return edge_eval(x, V3{cur[0], cur[1], cur[2]}, V3{a[0], a[1], a[2]}, V3{b[0], b[1], b[2]}, weight, J);
}

double pfref_surf_eval(const double x[7], const double cur[3], const double n[3], double d, double weight,
                       double J[7]) {
    return surf_eval(x, V3{cur[0], cur[1], cur[2]}, V3{n[0], n[1], n[2]}, d, weight, J);
}

static pfref_odom* create(const pfref_lidar* lidar, const pfref_odom_params* p, int opts, bool bpf) {
    if (!(p->weight_type == 0 || p->weight_type == 1 || p->weight_type == 2 || p->weight_type == 12)) return nullptr;
    pfref_odom* h = new pfref_odom();
    Odom& o = h->o;
    o.lidar = *lidar;
    o.opts = opts;
    o.map_resolution = (float)p->map_resolution;
    // ES (:186-190): corner leaf r, surf leaf 2r. BPF (:657-659): beam r, pillar r, facade 2r.
    o.nc = bpf ? 3 : 2;
    for (int c = 0; c < o.nc; ++c) {
        o.plane[c] = c == o.nc - 1;
        o.leaf_vg[c] = o.plane[c] ? (float)(p->map_resolution * 2) : (float)p->map_resolution;  // double -> float
        o.leaf_rg[c] = o.plane[c] ? o.map_resolution * 2 : o.map_resolution;                    // float
    }
    o.odom = iso_identity();
    o.last_odom = iso_identity();
    o.optimization_count = 2;
    o.k_new_surf = o.k_new_edge = p->k_new;
    o.theta_p_surf = o.theta_p_edge = p->theta_p;
    o.theta_max_surf = o.theta_max_edge = p->theta_max;
    o.weightType = p->weight_type;
    return h;
}

pfref_odom* pfref_odom_create(const pfref_lidar* lidar, const pfref_odom_params* p, int opts) {
    return create(lidar, p, opts, false);
}
pfref_odom* pfref_bpf_create(const pfref_lidar* lidar, const pfref_odom_params* p, int opts) {
    return create(lidar, p, opts, true);
}

void pfref_odom_destroy(pfref_odom* h) { delete h; }

int pfref_odom_classes(const pfref_odom* h) { return h->o.nc; }

// initMapWithPoints (ES :217-222, BPF :685-691): append the raw clouds, optimization_count = 12
int pfref_odom_init_map_n(pfref_odom* h, const float* const* clouds, const size_t* n) {
    Odom& o = h->o;
    o.stats = pfref_stats{};
    for (int c = 0; c < o.nc; ++c) {
        std::vector<PtC> v = to_ptc(clouds[c], n[c]);
        o.maps[c].insert(o.maps[c].end(), v.begin(), v.end());
        o.stats.n_in[c] = (int64_t)n[c];
        o.stats.n_map[c] = (int64_t)o.maps[c].size();
    }
    o.optimization_count = 12;
    h->inited = true;
    legacy_stats(o);
    return 0;
}

int pfref_odom_init_map(pfref_odom* h, const float* edge, size_t ne, const float* surf, size_t ns) {
    const float* c[2] = {edge, surf};
    const size_t n[2] = {ne, ns};
    return pfref_odom_init_map_n(h, c, n);
}

void pfref_odom_get_pose(const pfref_odom* h, double pose[7]) {
    Quat q = m2q(rotation_polar(h->o.odom.R));  // q_current(odom.rotation()) in the node (copy.cpp:105)
    pose[0] = q.x; pose[1] = q.y; pose[2] = q.z; pose[3] = q.w;
    pose[4] = h->o.odom.t.x; pose[5] = h->o.odom.t.y; pose[6] = h->o.odom.t.z;
}

int pfref_odom_update_n(pfref_odom* h, const float* const* clouds, const size_t* n, double pose_out[7]) {
    std::vector<PtC> in[3];
    for (int c = 0; c < h->o.nc; ++c) in[c] = to_ptc(clouds[c], n[c]);
    int rc = odom_update(h->o, in);
    if (pose_out) pfref_odom_get_pose(h, pose_out);
    return rc;
}

int pfref_odom_update(pfref_odom* h, const float* edge, size_t ne, const float* surf, size_t ns, double pose_out[7]) {
    const float* c[2] = {edge, surf};
    const size_t n[2] = {ne, ns};
    return pfref_odom_update_n(h, c, n, pose_out);
}

int pfref_odom_get_map(const pfref_odom* h, int which, float* xyz, uint8_t* rg, size_t cap, size_t* n) {
    if (which < 0 || which >= h->o.nc) return -1;
    const std::vector<PtC>& m = h->o.maps[which];
    *n = m.size();
    if (m.size() > cap) return -1;
    for (size_t i = 0; i < m.size(); ++i) {
        if (xyz) { xyz[3 * i] = m[i].x; xyz[3 * i + 1] = m[i].y; xyz[3 * i + 2] = m[i].z; }
        if (rg) { rg[2 * i] = m[i].r; rg[2 * i + 1] = m[i].g; }
    }
    return 0;
}

int pfref_odom_set_map(pfref_odom* h, int which, const float* xyz, const uint8_t* rg, size_t n) {
    if (which < 0 || which >= h->o.nc) return -1;
    std::vector<PtC>& m = h->o.maps[which];
    m.resize(n);
    for (size_t i = 0; i < n; ++i) {
        m[i].x = xyz[3 * i]; m[i].y = xyz[3 * i + 1]; m[i].z = xyz[3 * i + 2];
        m[i].r = rg ? rg[2 * i] : 0; m[i].g = rg ? rg[2 * i + 1] : 0; m[i].b = 0;
    }
    return 0;
}

void pfref_odom_get_stats(const pfref_odom* h, pfref_stats* s) { *s = h->o.stats; }

void pfref_odom_set_state(pfref_odom* h, const double odom_pose[7], const double last_pose[7]) {
    Quat q{odom_pose[0], odom_pose[1], odom_pose[2], odom_pose[3]};
    h->o.odom.R = q2m(q);
    h->o.odom.t = V3{odom_pose[4], odom_pose[5], odom_pose[6]};
    Quat ql{last_pose[0], last_pose[1], last_pose[2], last_pose[3]};
    h->o.last_odom.R = q2m(ql);
    h->o.last_odom.t = V3{last_pose[4], last_pose[5], last_pose[6]};
    for (int k = 0; k < 7; ++k) h->o.params[k] = odom_pose[k];
    h->inited = true;                                   // the next frame runs updatePointsToMap
}

void pfref_odom_set_opt_count(pfref_odom* h, int n) { h->o.optimization_count = n; }

int pfref_odom_frame(pfref_odom* h, const pfref_lidar* lidar, const float* xyzi, size_t n, double pose_out[7]) {
    if (h->o.nc != 2) return -1;                       // featureExtraction feeds the ES estimator only
    std::vector<PtI> e, s;
    feature_extraction(*lidar, h->o.opts, reinterpret_cast<const PtI*>(xyzi), n, e, s);
    const float* ep = reinterpret_cast<const float*>(e.data());
    const float* sp = reinterpret_cast<const float*>(s.data());
    if (!h->inited) {                                   // odomEstimationNode copy.cpp:87-90
        int rc = pfref_odom_init_map(h, ep, e.size(), sp, s.size());
        if (pose_out) pfref_odom_get_pose(h, pose_out);
        return rc;
    }
    return pfref_odom_update(h, ep, e.size(), sp, s.size(), pose_out);
}

}  // extern "C"
