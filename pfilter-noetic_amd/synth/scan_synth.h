/* Deterministic synthetic LiDAR workload generator (S64 / S32 / S128 scans and
 * the 2M-point dense urban map of BASELINE config 5).
 *
 * This is workload input for tests and bench.py, not part of the odometry hot
 * path. The scene model follows SURVEY.md §8(d): ground plane 1.73 m below the
 * sensor, box buildings set back from a curving road, poles and parked cars (S64V adds
 * porous tree crowns, trunks and hedges and a rough ground height field),
 * ray-cast per beam/azimuth with N(0, 0.02 m) range noise and random dropout.
 * Points are emitted azimuth-major (all beams of one azimuth step, then the
 * next), so each ring is in azimuth order, as in a Velodyne sweep.
 */
#ifndef PF_SCAN_SYNTH_H
#define PF_SCAN_SYNTH_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int lines;              /* 64, 32 or 128 */
    int az_steps;           /* azimuth steps per revolution */
    double speed;           /* m/s */
    double scan_period;     /* s */
    double yaw_amp;         /* rad/s amplitude of the yaw-rate sinusoid */
    double yaw_period;      /* s */
    double dropout;         /* fraction of rays dropped */
    double range_noise;     /* sigma, m */
    double max_range;       /* m */
    double sensor_height;   /* m above ground */
    double building_prob;   /* probability a building slot is filled */
    double setback_min, setback_max;
    int seed;
    double vegetation;      /* 0: none; > 0: trees / hedges per metre of road (porous volumes) */
    double terrain;         /* amplitude (m) of the rough-ground height field (0: flat) */
    double cross;           /* 0: none; > 0: cross streets, walls across the road and landmarks off the
                               road axis per metre of road (S64T) */
} pfsyn_params;

/* preset 0: S64 KITTI-like (config 1/2/4), 1: S32 campus (config 3), 2: S128 (config 5),
 * 3: S64V, S64 in a residential scene with vegetation and rough ground (KITTI-00 density),
 * 4: S64T, a well-conditioned town: turns, cross streets, walls across the road and landmarks off
 *    the road axis, so every direction of the pose is observed (the free-running parity scene) */
void pfsyn_default_params(int preset, pfsyn_params* p);

/* Builds the world along the trajectory for n_frames frames. Returns NULL on error. */
void* pfsyn_create(const pfsyn_params* p, int n_frames);
void pfsyn_destroy(void* h);
int pfsyn_num_frames(void* h);

/* Ray-casts one frame. xyzi_out holds 4 floats per point (x, y, z, intensity) in the
 * sensor frame. ring_out (optional) receives the beam index of every point.
 * Returns 0 on success, -1 if cap is too small. */
int pfsyn_frame(void* h, int frame, float* xyzi_out, size_t cap, size_t* n_out, int* ring_out);

/* Ray-casts frames [f0, f0+nf) using up to `threads` OpenMP threads. Frame k is written
 * at out + k*cap_per_frame*4 floats; counts[k] receives its point count. */
int pfsyn_frames(void* h, int f0, int nf, float* out, size_t cap_per_frame, size_t* counts, int threads);

/* Ground-truth pose of the sensor at `frame`, relative to frame 0:
 * pose = {qx, qy, qz, qw, tx, ty, tz}. */
void pfsyn_gt_pose(void* h, int frame, double pose[7]);

/* Config-5 dense urban block: n points (x, y, z, 0) written to xyz4 (4 floats each),
 * surface samples of ground, facades and floor slabs within a 200 m block. */
int pfsyn_dense_map(int seed, size_t n, float* xyz4);

/* Config-5 queries: points near the dense map's surfaces with N(0, sigma) jitter. */
int pfsyn_dense_queries(int seed, size_t nq, double sigma, const float* map_xyz4, size_t nmap,
                        float* q_xyz4);

#ifdef __cplusplus
}
#endif
#endif
