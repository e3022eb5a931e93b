// Deterministic synthetic LiDAR scene + ray caster (workload input; see scan_synth.h).
#include "scan_synth.h"

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
inline uint64_t key4(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    return mix64(mix64(mix64(mix64(a) ^ b) ^ c) ^ d);
}

struct Rng {  // sequential generator for world building
    uint64_t s;
    explicit Rng(uint64_t seed) : s(mix64(seed ^ 0x5bd1e995ull)) {}
    double u() { s = mix64(s); return u01(s); }
    double u(double a, double b) { return a + (b - a) * u(); }
};

struct Box { double cx, cy, c, s, hx, hy, z0, z1, br, pen; uint64_t key; };   // pen > 0: porous (hedge)
struct Cyl { double cx, cy, r, z0, z1; };
struct Sph { double cx, cy, cz, r; uint64_t key; };               // porous tree crown
constexpr double kCrownPen = 0.35;                                // mean penetration depth into foliage (m)
constexpr int kSphBase = 1 << 28;                                 // primitive ids >= kSphBase: crowns

struct PathSample { double x, y, psi; };

struct World {
    pfsyn_params p;
    int n_frames;
    double ds;              // path sample spacing (m)
    double s0;              // arc length of sample 0
    std::vector<PathSample> path;
    std::vector<Box> boxes;
    std::vector<Cyl> cyls;
    std::vector<Sph> sphs;
    std::vector<double> elev;  // beam elevations (rad)

    double heading_at_time(double t) const {
        if (t <= 0) return 0.0;
        const double P = p.yaw_period, A = p.yaw_amp;
        return A * P / (2.0 * M_PI) * (1.0 - std::cos(2.0 * M_PI * t / P));
    }
    PathSample at_s(double s) const {
        double fi = (s - s0) / ds;
        if (fi < 0) fi = 0;
        size_t i = (size_t)fi;
        if (i + 1 >= path.size()) return path.back();
        double w = fi - (double)i;
        const PathSample& a = path[i];
        const PathSample& b = path[i + 1];
        return {a.x + w * (b.x - a.x), a.y + w * (b.y - a.y), a.psi + w * (b.psi - a.psi)};
    }
};

void build_path(World& w) {
    const double v = w.p.speed > 0 ? w.p.speed : 1.0;
    const double T = w.n_frames * w.p.scan_period;
    const double pre = 250.0, post = 250.0;  // metres of road before/after
    w.ds = 0.25;
    w.s0 = -pre;
    size_t n = (size_t)((pre + v * T + post) / w.ds) + 2;
    w.path.resize(n);
    // backwards straight segment, then integrate forward (midpoint rule, 10 substeps)
    size_t i0 = (size_t)(pre / w.ds);
    for (size_t i = 0; i <= i0; ++i) {
        double s = w.s0 + i * w.ds;
        w.path[i] = {s, 0.0, 0.0};
    }
    double x = 0, y = 0;
    w.path[i0] = {0, 0, 0};
    for (size_t i = i0 + 1; i < n; ++i) {
        double s_prev = (i - 1 - i0) * w.ds;
        const int sub = 10;
        double h = w.ds / sub;
        for (int k = 0; k < sub; ++k) {
            double sm = s_prev + (k + 0.5) * h;
            double psi = w.heading_at_time(sm / v);
            x += h * std::cos(psi);
            y += h * std::sin(psi);
        }
        double s = (i - i0) * w.ds;
        w.path[i] = {x, y, w.heading_at_time(s / v)};
    }
}

// a porous object's hash key from its position (not its index: the scene of a longer sequence has
// more objects, and a prefix must stay the same scene)
inline uint64_t obj_key(double cx, double cy) {
    uint64_t a, b;
    std::memcpy(&a, &cx, 8);
    std::memcpy(&b, &cy, 8);
    return mix64(a ^ mix64(b));
}

void add_box(World& w, double cx, double cy, double psi, double hx, double hy, double z0, double z1,
             double pen = 0.0) {
    Box b;
    b.cx = cx; b.cy = cy; b.c = std::cos(psi); b.s = std::sin(psi);
    b.hx = hx; b.hy = hy; b.z0 = z0; b.z1 = z1;
    b.br = std::sqrt(hx * hx + hy * hy);
    b.pen = pen;
    b.key = obj_key(cx, cy);
    w.boxes.push_back(b);
}

// One RNG stream per (side, object kind): the objects laid along the road depend only on the seed
// and the arc length, never on how many frames the sequence has (a prefix of a longer sequence is
// the same scene).
void build_scene(World& w) {
    const double s_begin = w.s0 + 5.0;
    const double s_end = w.s0 + (w.path.size() - 2) * w.ds;
    for (int side = -1; side <= 1; side += 2) {
        const uint64_t base = (uint64_t)w.p.seed * 7919ull + 17ull + (side > 0 ? 100ull : 0ull);
        Rng rng(base);
        // buildings
        double s = s_begin + rng.u(0.0, 10.0);
        while (s < s_end) {
            double L = rng.u(6.0, 16.0);
            double gap = rng.u(1.0, 5.0);
            if (w.p.cross > 0 && rng.u() < 0.25) gap += rng.u(12.0, 25.0);       // a cross street
            if (rng.u() < w.p.building_prob) {
                double sm = s + 0.5 * L;
                PathSample ps = w.at_s(sm);
                double setback = rng.u(w.p.setback_min, w.p.setback_max);
                double depth = rng.u(8.0, 20.0);
                double hu = rng.u();
                double height = 2.0 + 23.0 * hu * hu;
                double nx = -std::sin(ps.psi), ny = std::cos(ps.psi);
                double off = side * (setback + 0.5 * depth);
                add_box(w, ps.x + nx * off, ps.y + ny * off, ps.psi, 0.5 * L, 0.5 * depth, 0.0, height);
            }
            s += L + gap;
        }
        // poles
        rng = Rng(base + 1);
        s = s_begin + rng.u(0.0, 5.0);
        while (s < s_end) {
            PathSample ps = w.at_s(s);
            double lat = rng.u(4.0, 5.5) * side;
            Cyl c;
            c.cx = ps.x - std::sin(ps.psi) * lat;
            c.cy = ps.y + std::cos(ps.psi) * lat;
            c.r = rng.u(0.1, 0.2);
            c.z0 = 0.0;
            c.z1 = rng.u(3.0, 8.0);
            w.cyls.push_back(c);
            s += rng.u(5.0, 10.0);
        }
        // parked cars
        rng = Rng(base + 2);
        s = s_begin + rng.u(0.0, 10.0);
        while (s < s_end) {
            if (rng.u() < 0.5) {
                PathSample ps = w.at_s(s);
                double lat = rng.u(3.0, 3.6) * side;
                double psi = ps.psi + rng.u(-0.05, 0.05);
                add_box(w, ps.x - std::sin(ps.psi) * lat, ps.y + std::cos(ps.psi) * lat, psi, 2.2, 0.9, 0.25, 1.5);
            }
            s += rng.u(6.0, 20.0);
        }
        if (w.p.cross > 0) {
            // walls and buildings across the road axis (their broad faces look along the road)
            rng = Rng(base + 6);
            s = s_begin + rng.u(0.0, 20.0);
            while (s < s_end) {
                PathSample ps = w.at_s(s);
                double lat = rng.u(10.0, 40.0) * side;
                double hx = rng.u(3.0, 8.0), hy = rng.u(0.3, 4.0), top = rng.u(2.5, 12.0);
                add_box(w, ps.x - std::sin(ps.psi) * lat, ps.y + std::cos(ps.psi) * lat,
                        ps.psi + 0.5 * M_PI + rng.u(-0.3, 0.3), hx, hy, 0.0, top);
                s += rng.u(20.0, 50.0) / w.p.cross;
            }
            // landmarks scattered off the road axis: posts, lamp masts, tree trunks
            rng = Rng(base + 7);
            s = s_begin + rng.u(0.0, 8.0);
            while (s < s_end) {
                PathSample ps = w.at_s(s);
                double lat = rng.u(6.0, 45.0) * side;
                Cyl c;
                c.cx = ps.x - std::sin(ps.psi) * lat;
                c.cy = ps.y + std::cos(ps.psi) * lat;
                c.r = rng.u(0.2, 0.6);
                c.z0 = 0.0;
                c.z1 = rng.u(2.0, 9.0);
                w.cyls.push_back(c);
                s += rng.u(6.0, 15.0) / w.p.cross;
            }
        }
        if (w.p.vegetation <= 0) continue;
        // trees: a trunk and a porous crown, spacing shrinking with the vegetation density
        rng = Rng(base + 3);
        s = s_begin + rng.u(0.0, 6.0);
        while (s < s_end) {
            PathSample ps = w.at_s(s);
            double lat = rng.u(5.5, 16.0) * side;
            double cx = ps.x - std::sin(ps.psi) * lat, cy = ps.y + std::cos(ps.psi) * lat;
            double r = rng.u(1.5, 3.5);
            double cz = rng.u(2.5, 5.5) + 0.5 * r;
            Cyl t;
            t.cx = cx; t.cy = cy; t.r = rng.u(0.12, 0.3); t.z0 = 0.0; t.z1 = cz - 0.5 * r;
            w.cyls.push_back(t);
            w.sphs.push_back(Sph{cx, cy, cz, r, obj_key(cx, cy)});
            s += rng.u(4.0, 12.0) / w.p.vegetation;
        }
        // the wooded background behind the kerb-side row (yards, parks): crowns only, denser
        rng = Rng(base + 5);
        s = s_begin + rng.u(0.0, 3.0);
        while (s < s_end) {
            PathSample ps = w.at_s(s);
            double lat = rng.u(16.0, 60.0) * side;
            double r = rng.u(2.0, 5.0);
            double cz = rng.u(3.0, 8.0) + 0.5 * r;
            double cx = ps.x - std::sin(ps.psi) * lat, cy = ps.y + std::cos(ps.psi) * lat;
            Cyl t;
            t.cx = cx; t.cy = cy; t.r = rng.u(0.15, 0.4); t.z0 = 0.0; t.z1 = cz - 0.5 * r;
            w.cyls.push_back(t);
            w.sphs.push_back(Sph{cx, cy, cz, r, obj_key(cx, cy)});
            s += rng.u(2.0, 6.0) / w.p.vegetation;
        }
        // hedges and bushes along the kerb: porous boxes
        rng = Rng(base + 4);
        s = s_begin + rng.u(0.0, 8.0);
        while (s < s_end) {
            double L = rng.u(2.0, 10.0);
            if (rng.u() < 0.6 * std::min(1.0, w.p.vegetation)) {
                PathSample ps = w.at_s(s + 0.5 * L);
                double lat = rng.u(4.5, 7.0) * side;
                add_box(w, ps.x - std::sin(ps.psi) * lat, ps.y + std::cos(ps.psi) * lat, ps.psi + rng.u(-0.1, 0.1),
                        0.5 * L, 0.5 * rng.u(0.6, 1.5), 0.0, rng.u(0.6, 1.8), 0.25);
            }
            s += L + rng.u(3.0, 15.0);
        }
    }
}

// rough ground: bilinear value noise on a 0.7 m lattice, amplitude p.terrain
double terrain_h(const World& w, double x, double y) {
    const double g = 0.7;
    const double fx = std::floor(x / g), fy = std::floor(y / g);
    const double ax = x / g - fx, ay = y / g - fy;
    auto v = [&](double i, double j) {
        return 2.0 * u01(key4((uint64_t)w.p.seed, (uint64_t)(int64_t)i, (uint64_t)(int64_t)j, 77)) - 1.0;
    };
    const double a = v(fx, fy) * (1 - ax) + v(fx + 1, fy) * ax;
    const double b = v(fx, fy + 1) * (1 - ax) + v(fx + 1, fy + 1) * ax;
    return w.p.terrain * (a * (1 - ay) + b * ay);
}

void build_beams(World& w) {
    w.elev.clear();
    const double d2r = M_PI / 180.0;
    if (w.p.lines == 64) {
        for (int k = 0; k < 32; ++k) w.elev.push_back((2.0 - (k + 0.1) / 3.0) * d2r);
        for (int k = 0; k < 32; ++k) w.elev.push_back((-8.83 - (k - 0.1) / 2.0) * d2r);
    } else if (w.p.lines == 32) {
        for (int k = 0; k < 32; ++k) w.elev.push_back((-92.0 / 3.0 + (k + 0.5) * 4.0 / 3.0) * d2r);
    } else if (w.p.lines == 16) {
        for (int k = 0; k < 16; ++k) w.elev.push_back((-15.0 + 2.0 * k + 0.1) * d2r);
    } else {
        int L = w.p.lines;
        for (int k = 0; k < L; ++k) w.elev.push_back((15.0 - 40.0 * (k + 0.5) / L) * d2r);
    }
}

inline bool hit_box(const Box& b, double ox, double oy, double oz, double dx, double dy, double dz,
                    double& t, uint64_t hash = 0) {
    double px = ox - b.cx, py = oy - b.cy;
    double lx = b.c * px + b.s * py, ly = -b.s * px + b.c * py;
    double ux = b.c * dx + b.s * dy, uy = -b.s * dx + b.c * dy;
    double t0 = 1e-3, t1 = 1e30;
    auto slab = [&](double o, double d, double lo, double hi) -> bool {
        if (std::fabs(d) < 1e-15) return o >= lo && o <= hi;
        double a = (lo - o) / d, c = (hi - o) / d;
        if (a > c) std::swap(a, c);
        if (a > t0) t0 = a;
        if (c < t1) t1 = c;
        return t0 <= t1;
    };
    if (!slab(lx, ux, -b.hx, b.hx)) return false;
    if (!slab(ly, uy, -b.hy, b.hy)) return false;
    if (!slab(oz, dz, b.z0, b.z1)) return false;
    if (b.pen > 0) {                        // porous: the ray stops inside or passes through
        const double d = -std::log(std::max(u01(hash), 1e-300)) * b.pen;
        if (t0 + d > t1) return false;
        t = t0 + d;
        return true;
    }
    t = t0;
    return true;
}

inline bool hit_sph(const Sph& c, double ox, double oy, double oz, double dx, double dy, double dz, double& t,
                    uint64_t hash) {
    const double px = ox - c.cx, py = oy - c.cy, pz = oz - c.cz;
    const double B = px * dx + py * dy + pz * dz;            // |d| = 1
    const double C = px * px + py * py + pz * pz - c.r * c.r;
    const double disc = B * B - C;
    if (disc < 0) return false;
    const double sq = std::sqrt(disc);
    const double t0 = std::max(-B - sq, 1e-3), t1 = -B + sq;
    if (t1 <= t0) return false;
    const double d = -std::log(std::max(u01(hash), 1e-300)) * kCrownPen;
    if (t0 + d > t1) return false;          // through a gap in the foliage
    t = t0 + d;
    return true;
}

inline bool hit_cyl(const Cyl& c, double ox, double oy, double oz, double dx, double dy, double dz,
                    double& t) {
    double px = ox - c.cx, py = oy - c.cy;
    double A = dx * dx + dy * dy;
    if (A < 1e-18) return false;
    double B = px * dx + py * dy;
    double C = px * px + py * py - c.r * c.r;
    double disc = B * B - A * C;
    if (disc < 0) return false;
    double tt = (-B - std::sqrt(disc)) / A;
    if (tt <= 1e-3) return false;
    double z = oz + tt * dz;
    if (z < c.z0 || z > c.z1) return false;
    t = tt;
    return true;
}

constexpr int NBINS = 720;

size_t cast_frame(const World& w, int frame, float* out, size_t cap, int* ring_out, bool* overflow) {
    const pfsyn_params& p = w.p;
    const double t = frame * p.scan_period;
    const PathSample ps = w.at_s(p.speed * t);
    const double sx = ps.x, sy = ps.y, sz = p.sensor_height, psi = ps.psi;
    const double cpsi = std::cos(psi), spsi = std::sin(psi);

    // azimuth binning of primitives (index >= 0: box, < 0: ~cylinder)
    std::vector<std::vector<int>> bins(NBINS);
    auto add_interval = [&](int id, double bx, double by, double br) {
        double dxw = bx - sx, dyw = by - sy;
        double dist = std::sqrt(dxw * dxw + dyw * dyw);
        if (dist - br > p.max_range) return;
        if (dist <= br + 1e-6) {
            for (int b = 0; b < NBINS; ++b) bins[b].push_back(id);
            return;
        }
        double th = std::atan2(dyw, dxw) - psi;
        double al = std::asin(std::min(1.0, br / dist)) + 1e-3;
        int b0 = (int)std::floor((th - al + M_PI) / (2 * M_PI) * NBINS);
        int b1 = (int)std::floor((th + al + M_PI) / (2 * M_PI) * NBINS);
        if (b1 - b0 >= NBINS) { b0 = 0; b1 = NBINS - 1; }
        for (int b = b0; b <= b1; ++b) bins[((b % NBINS) + NBINS) % NBINS].push_back(id);
    };
    for (size_t i = 0; i < w.boxes.size(); ++i)
        add_interval((int)i, w.boxes[i].cx, w.boxes[i].cy, w.boxes[i].br);
    for (size_t i = 0; i < w.cyls.size(); ++i)
        add_interval(~(int)i, w.cyls[i].cx, w.cyls[i].cy, w.cyls[i].r);
    for (size_t i = 0; i < w.sphs.size(); ++i)
        add_interval(kSphBase + (int)i, w.sphs[i].cx, w.sphs[i].cy, w.sphs[i].r);

    const int L = (int)w.elev.size();
    size_t n = 0;
    for (int k = 0; k < p.az_steps; ++k) {
        // sweep starts behind the sensor, counter-clockwise
        double az = -M_PI + (k + 0.5) * (2.0 * M_PI / p.az_steps);
        int bin = (int)std::floor((az + M_PI) / (2 * M_PI) * NBINS);
        if (bin >= NBINS) bin = NBINS - 1;
        if (bin < 0) bin = 0;
        const std::vector<int>& cand = bins[bin];
        const double ca = std::cos(az), sa = std::sin(az);
        for (int b = 0; b < L; ++b) {
            uint64_t ray = (uint64_t)k * 1024u + (uint64_t)b;
            uint64_t h0 = key4((uint64_t)p.seed, (uint64_t)frame, ray, 1);
            if (u01(h0) < p.dropout) continue;
            double ce = std::cos(w.elev[b]), se = std::sin(w.elev[b]);
            double lx = ce * ca, ly = ce * sa, lz = se;       // sensor-frame direction
            double dx = cpsi * lx - spsi * ly, dy = spsi * lx + cpsi * ly, dz = lz;
            double best = p.max_range;
            bool hit = false;
            if (dz < -1e-12) {
                double tg = -sz / dz;
                if (p.terrain > 0) {            // one fixed-point step onto the height field
                    const double h = terrain_h(w, sx + tg * dx, sy + tg * dy);
                    tg = (h - sz) / dz;
                }
                if (tg > 0 && tg < best) { best = tg; hit = true; }
            }
            for (int id : cand) {
                double th;
                if (id >= kSphBase) {
                    const uint64_t hs = key4((uint64_t)p.seed, (uint64_t)frame, ray, w.sphs[id - kSphBase].key);
                    if (hit_sph(w.sphs[id - kSphBase], sx, sy, sz, dx, dy, dz, th, hs) && th < best) { best = th; hit = true; }
                } else if (id >= 0) {
                    const uint64_t hs = w.boxes[id].pen > 0 ? key4((uint64_t)p.seed, (uint64_t)frame, ray, w.boxes[id].key) : 0;
                    if (hit_box(w.boxes[id], sx, sy, sz, dx, dy, dz, th, hs) && th < best) { best = th; hit = true; }
                } else {
                    if (hit_cyl(w.cyls[~id], sx, sy, sz, dx, dy, dz, th) && th < best) { best = th; hit = true; }
                }
            }
            if (!hit) continue;
            uint64_t h1 = key4((uint64_t)p.seed, (uint64_t)frame, ray, 2);
            uint64_t h2 = key4((uint64_t)p.seed, (uint64_t)frame, ray, 3);
            uint64_t h3 = key4((uint64_t)p.seed, (uint64_t)frame, ray, 4);
            double u1 = std::max(u01(h1), 1e-300), u2 = u01(h2);
            double g = std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
            double r = best + p.range_noise * g;
            if (r <= 0.05) continue;
            if (n >= cap) { *overflow = true; return n; }
            out[4 * n + 0] = (float)(r * lx);
            out[4 * n + 1] = (float)(r * ly);
            out[4 * n + 2] = (float)(r * lz);
            out[4 * n + 3] = (float)u01(h3);
            if (ring_out) ring_out[n] = b;
            ++n;
        }
    }
    return n;
}

}  // namespace

extern "C" {

void pfsyn_default_params(int preset, pfsyn_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->scan_period = 0.1;
    p->dropout = 0.06;
    p->range_noise = 0.02;
    p->max_range = 120.0;
    p->sensor_height = 1.73;
    p->yaw_amp = 0.1;
    p->yaw_period = 60.0;
    if (preset == 1) {          // S32 campus, slow
        p->lines = 32; p->az_steps = 1800; p->speed = 2.0; p->seed = 2;
        p->building_prob = 0.5; p->setback_min = 10.0; p->setback_max = 30.0;
    } else if (preset == 2) {   // S128
        p->lines = 128; p->az_steps = 1563; p->speed = 10.0; p->seed = 5;
        p->building_prob = 0.85; p->setback_min = 6.0; p->setback_max = 20.0;
    } else if (preset == 3) {   // S64V: residential, vegetation and rough ground (KITTI-00 density)
        p->lines = 64; p->az_steps = 2000; p->speed = 8.0; p->seed = 0;
        p->building_prob = 0.35; p->setback_min = 8.0; p->setback_max = 30.0;
        p->vegetation = 1.0; p->terrain = 0.08;
    } else if (preset == 4) {   // S64T: the well-conditioned town
        p->lines = 64; p->az_steps = 2000; p->speed = 10.0; p->seed = 0;
        p->building_prob = 0.35; p->setback_min = 10.0; p->setback_max = 35.0;
        p->yaw_amp = 0.2; p->yaw_period = 40.0;
        p->cross = 1.0;
    } else {                    // S64 KITTI-like
        p->lines = 64; p->az_steps = 2000; p->speed = 10.0; p->seed = 0;
        p->building_prob = 0.85; p->setback_min = 6.0; p->setback_max = 20.0;
    }
}

void* pfsyn_create(const pfsyn_params* p, int n_frames) {
    if (!p || n_frames <= 0 || p->az_steps <= 0 || p->lines <= 0) return nullptr;
    World* w = new World();
    w->p = *p;
    w->n_frames = n_frames;
    build_path(*w);
    build_scene(*w);
    build_beams(*w);
    return w;
}

void pfsyn_destroy(void* h) { delete static_cast<World*>(h); }

int pfsyn_num_frames(void* h) { return static_cast<World*>(h)->n_frames; }

int pfsyn_frame(void* h, int frame, float* xyzi_out, size_t cap, size_t* n_out, int* ring_out) {
    const World* w = static_cast<World*>(h);
    bool of = false;
    size_t n = cast_frame(*w, frame, xyzi_out, cap, ring_out, &of);
    *n_out = n;
    return of ? -1 : 0;
}

int pfsyn_frames(void* h, int f0, int nf, float* out, size_t cap_per_frame, size_t* counts, int threads) {
    const World* w = static_cast<World*>(h);
    int err = 0;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads) reduction(| : err)
#endif
    for (int k = 0; k < nf; ++k) {
        bool of = false;
        counts[k] = cast_frame(*w, f0 + k, out + (size_t)k * cap_per_frame * 4, cap_per_frame, nullptr, &of);
        if (of) err |= 1;
    }
    (void)threads;
    return err ? -1 : 0;
}

void pfsyn_gt_pose(void* h, int frame, double pose[7]) {
    const World* w = static_cast<World*>(h);
    const double t = frame * w->p.scan_period;
    PathSample ps = w->at_s(w->p.speed * t);
    pose[0] = 0.0;
    pose[1] = 0.0;
    pose[2] = std::sin(0.5 * ps.psi);
    pose[3] = std::cos(0.5 * ps.psi);
    pose[4] = ps.x;
    pose[5] = ps.y;
    pose[6] = 0.0;
}

int pfsyn_dense_map(int seed, size_t n, float* xyz4) {
    // Ground + multi-storey blocks (facades and floor slabs every 3 m), sampled on a
    // jittered 0.8 m lattice inside a 200 m x 200 m block, until n points exist.
    Rng rng((uint64_t)seed * 104729ull + 3ull);
    size_t k = 0;
    const double h = 0.8;
    auto emit = [&](double x, double y, double z) -> bool {
        if (k >= n) return false;
        xyz4[4 * k + 0] = (float)(x + rng.u(-0.1, 0.1));
        xyz4[4 * k + 1] = (float)(y + rng.u(-0.1, 0.1));
        xyz4[4 * k + 2] = (float)(z + rng.u(-0.05, 0.05));
        xyz4[4 * k + 3] = 0.0f;
        ++k;
        return true;
    };
    for (double x = -100.0; x < 100.0 && k < n; x += h)
        for (double y = -100.0; y < 100.0 && k < n; y += h) emit(x, y, -1.73);
    while (k < n) {
        double cx = rng.u(-90.0, 90.0), cy = rng.u(-90.0, 90.0);
        double hx = rng.u(5.0, 15.0), hy = rng.u(5.0, 15.0);
        double top = rng.u(10.0, 45.0);
        for (double z = -1.73 + 3.0; z < top && k < n; z += 3.0)           // slabs
            for (double x = cx - hx; x < cx + hx && k < n; x += h)
                for (double y = cy - hy; y < cy + hy && k < n; y += h) emit(x, y, z);
        for (double z = -1.73; z < top && k < n; z += h) {                  // facades
            for (double x = cx - hx; x < cx + hx && k < n; x += h) { emit(x, cy - hy, z); emit(x, cy + hy, z); }
            for (double y = cy - hy; y < cy + hy && k < n; y += h) { emit(cx - hx, y, z); emit(cx + hx, y, z); }
        }
    }
    return 0;
}

int pfsyn_dense_queries(int seed, size_t nq, double sigma, const float* map_xyz4, size_t nmap, float* q) {
    if (nmap == 0) return -1;
    for (size_t i = 0; i < nq; ++i) {
        // stratified over the map's (spatially coherent) emission order, like a scan
        uint64_t hsel = key4((uint64_t)seed, i, 11, 0);
        size_t j = (size_t)(((double)i + u01(hsel)) * (double)nmap / (double)nq);
        if (j >= nmap) j = nmap - 1;
        for (int d = 0; d < 3; ++d) {
            double u1 = std::max(u01(key4((uint64_t)seed, i, 12 + d, 0)), 1e-300);
            double u2 = u01(key4((uint64_t)seed, i, 22 + d, 0));
            double g = std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
            q[4 * i + d] = (float)(map_xyz4[4 * j + d] + sigma * g);
        }
        q[4 * i + 3] = 0.0f;
    }
    return 0;
}

}  // extern "C"
