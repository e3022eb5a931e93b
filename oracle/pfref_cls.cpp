// pfref: the BPF front end — groundSeg::ground_seg and nongroundExtract::featureExtract.
// TEST INFRASTRUCTURE (oracle) — see pfref.h header.
//
// Restates, in the order the reference evaluates them:
//   groundSeg::ground_seg            include/preProcess.hpp:398-505 (bounds :522-564, grid_t :6-29)
//   nongroundExtract::pc2pc          include/preProcess.hpp:633-644 (xyz only)
//   nongroundExtract::featureExtract include/preProcess.hpp:646-689
//   PrincipleComponentAnalysis::get_pc_pca_feature / get_pca_feature  :200-247, :283-323
// as the additionNode callback chains them (src/additionNode.cpp:21-45; the DCVC `curvedfilter`
// stage between them is not restated: SURVEY §8(f) rank 4).
//
// Third-party arithmetic (parity unpinned):
//   KdTreeFLANN::radiusSearch(i, r, idx, d2, k): the <= k nearest points with f32 d^2 < r^2
//     (x -> y -> z, no FMA), ascending; ties by index.
//   pcl::PCA: f32 centroid (sequential sum / n), f32 covariance of the demeaned points summed in
//     neighbour order (Eigen's product blocking is not reproduced), eigen-decomposition by the
//     oracle's f64 cyclic Jacobi of the f32 covariance rounded back to f32 (Eigen's f32
//     tridiagonal QL is not reproduced), eigenvalues descending, col(2) = col(0) x col(1).
#include "pfref_internal.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <unordered_map>

namespace pfref {
namespace {

struct P3 { float x, y, z; };

const P3* at(const float* base, size_t stride, size_t i) {
    return reinterpret_cast<const P3*>(reinterpret_cast<const char*>(base) + i * stride);
}

// ground_seg: (ground, unground) as indices into the input, in the reference's push order
void ground_seg(const float* pts, size_t n, size_t stride, const pfref_cls_params& p, std::vector<int>& ground,
                std::vector<int>& unground) {
    ground.clear();
    unground.clear();
    // get_cloud_bbx (:522-556): double bounds of the float coordinates
    double min_x = DBL_MAX, min_y = DBL_MAX, max_x = -DBL_MAX, max_y = -DBL_MAX;
    for (size_t i = 0; i < n; ++i) {
        const P3* q = at(pts, stride, i);
        if (min_x > q->x) min_x = q->x;
        if (min_y > q->y) min_y = q->y;
        if (max_x < q->x) max_x = q->x;
        if (max_y < q->y) max_y = q->y;
    }
    const double res = p.gf_grid_res;                                  // float parameter (:401)
    const int row = (int)std::ceil((max_y - min_y) / res);             // :413-415
    const int col = (int)std::ceil((max_x - min_x) / res);
    const long long num_grid = n ? (long long)row * col : 0;
    struct Cell { std::vector<int> ids; float min_z = FLT_MAX, nb_min_z = FLT_MAX; int count = 0; };
    std::vector<Cell> grid(num_grid > 0 ? (size_t)num_grid : 0);
    for (size_t j = 0; j < n; ++j) {                                   // :427-448
        const P3* q = at(pts, stride, j);
        const int tc = (int)std::floor((q->x - min_x) / res);
        const int tr = (int)std::floor((q->y - min_y) / res);
        const long long id = (long long)tr * col + tc;
        if (id < 0 || id >= num_grid) continue;
        Cell& c = grid[(size_t)id];
        c.count++;
        if (q->z > p.gf_max_ground_height) {
            unground.push_back((int)j);
        } else {
            c.ids.push_back((int)j);
            if (q->z < c.min_z && q->z > p.gf_min_ground_height) c.min_z = c.nb_min_z = q->z;
        }
    }
    for (long long m = 0; m < num_grid; ++m) {                         // :451-467
        const int r = (int)(m / col), cc = (int)(m % col);
        if (r >= 1 && r <= row - 2 && cc >= 1 && cc <= col - 2)
            for (int j = -1; j <= 1; ++j)
                for (int k = -1; k <= 1; ++k)
                    if (grid[m].nb_min_z > grid[m + j * col + k].min_z) grid[m].nb_min_z = grid[m + j * col + k].min_z;
    }
    for (long long i = 0; i < num_grid; ++i) {                         // :470-494
        const Cell& c = grid[i];
        if (c.count < p.gf_min_grid_pts) continue;
        if (c.min_z - c.nb_min_z < p.gf_neighbor_height_diff) {
            for (int id : c.ids) {
                const float z = at(pts, stride, (size_t)id)->z;
                if (z - c.min_z < p.gf_max_height_diff && z > p.gf_min_ground_height) ground.push_back(id);
                else unground.push_back(id);
            }
        } else {
            for (int id : c.ids) unground.push_back(id);
        }
    }
}

// 1 m hash grid for the radius search
struct CellGrid {
    std::unordered_map<uint64_t, std::vector<int>> cells;
    static uint64_t key(int x, int y, int z) {
        return ((uint64_t)(uint32_t)(x + (1 << 20)) << 42) | ((uint64_t)(uint32_t)(y + (1 << 20)) << 21) |
               (uint64_t)(uint32_t)(z + (1 << 20));
    }
    void build(const std::vector<P3>& c) {
        cells.clear();
        for (size_t i = 0; i < c.size(); ++i)
            cells[key((int)std::floor(c[i].x), (int)std::floor(c[i].y), (int)std::floor(c[i].z))].push_back((int)i);
    }
};

// KdTreeFLANN::radiusSearch(i, radius, idx, d2, k) (src: :218): the k nearest with d^2 < r^2
void radius_knn(const std::vector<P3>& c, const CellGrid& g, int i, float r2, int k,
                std::vector<std::pair<float, int>>& out) {
    out.clear();
    const P3 q = c[(size_t)i];
    const int cx = (int)std::floor(q.x), cy = (int)std::floor(q.y), cz = (int)std::floor(q.z);
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                auto it = g.cells.find(CellGrid::key(cx + dx, cy + dy, cz + dz));
                if (it == g.cells.end()) continue;
                for (int j : it->second) {
                    const P3& p = c[(size_t)j];
                    float d = 0.0f, t;
                    t = q.x - p.x; d += t * t;
                    t = q.y - p.y; d += t * t;
                    t = q.z - p.z; d += t * t;
                    if (d < r2) out.emplace_back(d, j);
                }
            }
    if ((int)out.size() > k) {
        std::partial_sort(out.begin(), out.begin() + k, out.end());
        out.resize((size_t)k);
    } else {
        std::sort(out.begin(), out.end());
    }
}

}  // namespace

// PCA of one point's neighbourhood and the featureExtract decision (:653-688): 0 none, 1 pillar,
// 2 beam, 3 facade (the reference's index_with_feature codes)
int pca_class(const std::vector<P3>& c, const std::vector<std::pair<float, int>>& nb, float qz,
              const pfref_cls_params& p, float* normal4 = nullptr) {
    const int n = (int)nb.size();
    if (normal4) normal4[0] = normal4[1] = normal4[2] = normal4[3] = 0.f;
    if (n <= 3) return 0;                                              // :289 (features zero-initialised, :206)
    float sx = 0.f, sy = 0.f, sz = 0.f;                                // compute3DCentroid
    for (const auto& e : nb) {
        sx += c[(size_t)e.second].x;
        sy += c[(size_t)e.second].y;
        sz += c[(size_t)e.second].z;
    }
    const float fn = (float)n;
    const float mx = sx / fn, my = sy / fn, mz = sz / fn;
    float cxx = 0.f, cxy = 0.f, cxz = 0.f, cyy = 0.f, cyz = 0.f, czz = 0.f;
    for (const auto& e : nb) {                                         // demeaned^T demeaned
        const float dx = c[(size_t)e.second].x - mx, dy = c[(size_t)e.second].y - my, dz = c[(size_t)e.second].z - mz;
        cxx += dx * dx; cxy += dx * dy; cxz += dx * dz;
        cyy += dy * dy; cyz += dy * dz; czz += dz * dz;
    }
    const double A[3][3] = {{cxx, cxy, cxz}, {cxy, cyy, cyz}, {cxz, cyz, czz}};
    double ev[3], V[3][3];
    eigen_sym3(A, ev, V);                                              // ascending
    // PCA order: descending values, col(i) = evd col(2 - i); col(2) = col(0) x col(1)
    const float l1 = (float)ev[2], l2 = (float)ev[1], l3 = (float)ev[0];
    float v0[3] = {(float)V[0][2], (float)V[1][2], (float)V[2][2]};
    const float v1[3] = {(float)V[0][1], (float)V[1][1], (float)V[2][1]};
    float nv[3] = {v0[1] * v1[2] - v0[2] * v1[1], v0[2] * v1[0] - v0[0] * v1[2], v0[0] * v1[1] - v0[1] * v1[0]};
    float sq = v0[0] * v0[0] + v0[1] * v0[1] + v0[2] * v0[2];           // normalize() (:305-306)
    if (sq > 0.f) { const float s = std::sqrt(sq); v0[0] /= s; v0[1] /= s; v0[2] /= s; }
    sq = nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2];
    if (sq > 0.f) { const float s = std::sqrt(sq); nv[0] /= s; nv[1] /= s; nv[2] /= s; }
    const double d1 = l1, d2 = l2, d3 = l3;                            // eigenvalue_t is double (:77-82)
    const double linear_2 = (d1 - d2) / d1;                            // :315-316
    const double planar_2 = (d2 - d3) / d1;
    // assign_normal (:327-346): get_pc_pca_feature gives every point with more than min_k = 1
    // neighbours the normal direction and planar_2 (:238-239, pt.normal[3] a float); featureExtract
    // then gives pillar / beam points the principal direction and linear_2 (:663-674)
    auto put = [&](const float* v, double w) {
        if (normal4) { normal4[0] = v[0]; normal4[1] = v[1]; normal4[2] = v[2]; normal4[3] = (float)w; }
    };
    put(nv, planar_2);
    if (!(n > p.k_min)) return 0;                                      // :657
    if (linear_2 > p.edge_thre) {                                      // :659-674
        if (std::fabs(v0[2]) > p.linear_vsin_high) { put(v0, linear_2); return 1; }
        if (std::fabs(v0[2]) < p.linear_vsin_low && qz < p.beam_h_max && qz > p.beam_h_min) { put(v0, linear_2); return 2; }
    } else if (planar_2 > p.planar_thre) {                             // :676-684
        if (std::fabs(nv[2]) < p.planar_vsin_low) return 3;
    }
    return 0;
}

}  // namespace pfref

using namespace pfref;

extern "C" {

void pfref_cls_default_params(pfref_cls_params* p) {
    p->ground_filter = 1;            // pfilter_kitti.launch:10 groundfilter
    p->gf_min_grid_pts = 8;          // include/preProcess.hpp:575 gf_grid_pt_num_thre
    p->gf_grid_res = 3.0f;           // :605
    p->gf_max_height_diff = 0.3f;    // :604 gf_max_grid_height_diff
    p->gf_neighbor_height_diff = 1.5f;  // :603
    p->gf_max_ground_height = 5.0f;  // :601
    p->gf_min_ground_height = -5.0f; // :602
    p->radius = 1.0f;                // :703 neighbor_searching_radius
    p->k = 25;                       // :705 neighbor_k
    p->k_min = 8;                    // :706 neigh_k_min
    p->edge_thre = 0.65f;            // :708
    p->planar_thre = 0.65f;          // :709
    p->linear_vsin_high = 0.94f;     // :710
    p->linear_vsin_low = 0.17f;      // :711
    p->planar_vsin_low = 0.34f;      // :713
    p->beam_h_max = FLT_MAX;         // :714
    p->beam_h_min = 0.5f;            // :715
}

int pfref_ground_seg(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, int32_t* ground,
                     size_t* ng, int32_t* unground, size_t* nu) {
    if (!p || (!xyz && n) || stride < 12) return -1;
    std::vector<int> g, u;
    ground_seg(xyz, n, stride, *p, g, u);
    if (ground) std::copy(g.begin(), g.end(), ground);
    if (unground) std::copy(u.begin(), u.end(), unground);
    if (ng) *ng = g.size();
    if (nu) *nu = u.size();
    return 0;
}

int pfref_pca_classify(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, uint8_t* cls,
                       int32_t* pt_num) {
    return pfref_pca_classify_normals(xyz, n, stride, p, cls, pt_num, nullptr);
}

int pfref_pca_classify_normals(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, uint8_t* cls,
                               int32_t* pt_num, float* normal4) {
    if (!p || (!xyz && n) || stride < 12 || p->k < 1) return -1;
    std::vector<P3> c(n);
    for (size_t i = 0; i < n; ++i) c[i] = *at(xyz, stride, i);
    CellGrid g;
    g.build(c);
    const float r2 = (float)((double)p->radius * (double)p->radius);
    std::vector<std::pair<float, int>> nb;
    for (size_t i = 0; i < n; ++i) {
        radius_knn(c, g, (int)i, r2, p->k, nb);
        if (pt_num) pt_num[i] = (int32_t)nb.size();
        const int code = pca_class(c, nb, c[i].z, *p, normal4 ? normal4 + 4 * i : nullptr);
        if (cls) cls[i] = (uint8_t)code;
    }
    return 0;
}

// the additionNode chain (groundfilter -> featurePreExtract): class clouds as input indices
// featureExtract on the points u (input indices, in that order): class clouds as input indices
static void classify_into(const float* xyz, size_t stride, const pfref_cls_params& p, const std::vector<int>& u,
                          int32_t* beam, size_t* nb, int32_t* pillar, size_t* np, int32_t* facade, size_t* nf) {
    std::vector<P3> c(u.size());
    for (size_t i = 0; i < u.size(); ++i) c[i] = *at(xyz, stride, (size_t)u[i]);
    CellGrid grid;
    grid.build(c);
    const float r2 = (float)((double)p.radius * (double)p.radius);
    std::vector<std::pair<float, int>> nbh;
    size_t cnt[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < c.size(); ++i) {
        radius_knn(c, grid, (int)i, r2, p.k, nbh);
        const int k = pca_class(c, nbh, c[i].z, p);
        int32_t* dst = k == 1 ? pillar : (k == 2 ? beam : (k == 3 ? facade : nullptr));
        if (k && dst) dst[cnt[k]] = u[i];
        cnt[k]++;
    }
    if (np) *np = cnt[1];
    if (nb) *nb = cnt[2];
    if (nf) *nf = cnt[3];
}

int pfref_bpf_preprocess(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, int32_t* beam,
                         size_t* nb, int32_t* pillar, size_t* np, int32_t* facade, size_t* nf, int32_t* ground,
                         size_t* ng) {
    if (!p || (!xyz && n) || stride < 12) return -1;
    std::vector<int> g, u;
    if (p->ground_filter) {
        ground_seg(xyz, n, stride, *p, g, u);
    } else {
        u.resize(n);
        for (size_t i = 0; i < n; ++i) u[i] = (int)i;
    }
    classify_into(xyz, stride, *p, u, beam, nb, pillar, np, facade, nf);
    if (ground) std::copy(g.begin(), g.end(), ground);
    if (ng) *ng = g.size();
    return 0;
}

int pfref_bpf_preprocess_dcvc(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p,
                              const pfref_dcvc_params* dp, int first_frame, int dcvc_mode, int32_t* beam, size_t* nb,
                              int32_t* pillar, size_t* np, int32_t* facade, size_t* nf, int32_t* ground,
                              size_t* ng) {
    if (!p || !dp || (!xyz && n) || stride < 12) return -1;
    std::vector<int> g, u;
    if (p->ground_filter) {
        ground_seg(xyz, n, stride, *p, g, u);
    } else {
        u.resize(n);
        for (size_t i = 0; i < n; ++i) u[i] = (int)i;
    }
    std::vector<float> uc(3 * (u.size() ? u.size() : 1));
    for (size_t i = 0; i < u.size(); ++i) {
        const P3* q = at(xyz, stride, (size_t)u[i]);
        uc[3 * i] = q->x; uc[3 * i + 1] = q->y; uc[3 * i + 2] = q->z;
    }
    std::vector<int32_t> kept(u.size() ? u.size() : 1);
    size_t nk = 0;
    if (pfref_dcvc_mode(uc.data(), u.size(), 12, dp, first_frame, dcvc_mode, kept.data(), &nk, nullptr)) return -1;
    std::vector<int> v(nk);
    for (size_t i = 0; i < nk; ++i) v[i] = u[(size_t)kept[i]];
    classify_into(xyz, stride, *p, v, beam, nb, pillar, np, facade, nf);
    if (ground) std::copy(g.begin(), g.end(), ground);
    if (ng) *ng = g.size();
    return 0;
}

}  // extern "C"
