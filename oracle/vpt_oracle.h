/*
 * vpt_oracle.h — CPU restatement of the reference integrator (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / the timed CPU baseline — never as a product path.
 * Every function restates a reference function and cites it (file:line under /root/reference).
 *
 * Pinning: the RNG (hash + pcg32_fast + uniform<float>) is pinned by the
 * KATs of SURVEY §8c and by oracle/_ref (pcg32_fast compiled from the reference's vendored header);
 * the blackbody table/lookup by the SURVEY §8c KATs.  NanoVDB (HDDA, Ray, Map, ReadAccessor,
 * trilinear sampler) and Eigen (summation orders) are absent from /root/reference and cannot be
 * built here: those parts follow their published semantics and are "parity unpinned".
 */
#ifndef VPT_ORACLE_H
#define VPT_ORACLE_H

#include <stdint.h>
#include "../include/vpt_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RNG (include/vpt/hash.hpp:20-67, include/vpt/random.hpp:86-115, pcg_random.hpp pcg32_fast) */
uint64_t vpto_hash(uint64_t seed, uint64_t jid);
void vpto_rng_u32(uint32_t seed, uint64_t jid, uint32_t* out, int n);
void vpto_rng_f32(uint32_t seed, uint64_t jid, float* out, int n);

/* Blackbody (src/precompute_blackbody.cpp, src/spectral.cpp).  cie = [471][3] floats (360..830 nm),
 * y_integral as in xyz.hpp:314.  Table is [500][3]. */
float vpto_planck(float lambda_m, float temperature_k);
void vpto_blackbody_table(const float* cie, float y_integral, float* out_500x3);
void vpto_blackbody_xyz(const float* table, const float* cie, float y_integral, float t, float* out3);

/* Grids: a NanoVDB-semantics tree built from a vpt_grid_desc (copied). */
typedef struct vpto_grid vpto_grid;
vpto_grid* vpto_grid_create(const vpt_grid_desc* desc);
void vpto_grid_destroy(vpto_grid* g);
/* fix_majorants_for_interpolation (src/volume.cpp:104-160), in place; returns leaf count. */
uint64_t vpto_grid_fix_majorants(vpto_grid* g);
void vpto_grid_leaf_max(const vpto_grid* g, float* out);
float vpto_grid_get_value(const vpto_grid* g, int32_t i, int32_t j, int32_t k);
uint32_t vpto_grid_get_dim(const vpto_grid* g, int32_t i, int32_t j, int32_t k);
/* Trilinear sample at an index-space point (SampleFromVoxels<Acc,1>). */
float vpto_grid_sample(const vpto_grid* g, float x, float y, float z);

/* Camera (src/camera.cpp:5-57, include/vpt/camera.hpp:14-23): world ray of raster (x,y)+jitter. */
void vpto_camera_ray(const vpt_configuration* cfg, int64_t x, int64_t y, float jx, float jy,
                     float* origin3, float* dir3);
/* Camera matrix: raster_to_world_dir linear (row-major 3x3) + translation. */
void vpto_camera_matrix(const vpt_configuration* cfg, float* lin9, float* trans3);

/* RayMajorantIterator trace of one world ray (volume.cpp:38-98): writes up to max_segments
 * (t0, t1, d_maj) triples; returns the number of segments (or -1 if the ray misses). */
int vpto_trace_segments(const vpto_grid* density, const float* origin3, const float* dir3,
                        float* out_segments, int max_segments);

/* Render jobs [jid_begin, jid_begin+jid_count) serially (the body of vpt::run, worker.cpp:104-207),
 * adding into film[H][W][4].  records (nullable): per-sample L as in vpt_gpu_render_jobs_records.
 * temperature may be NULL.  bb_table [500][3] (+cie for the T>=49900 K path). */
int vpto_render_jobs(const vpt_configuration* cfg, const vpto_grid* density,
                     const vpto_grid* temperature, const float* bb_table, const float* cie,
                     float y_integral, uint64_t jid_begin, uint64_t jid_count, float* film,
                     float* records, vpt_counters* counters);

/* Same with an RNG mode (VPT_RNG_REFERENCE / VPT_RNG_PIXEL, see vpt_gpu_set_rng_mode). */
int vpto_render_jobs_mode(const vpt_configuration* cfg, const vpto_grid* density,
                          const vpto_grid* temperature, const float* bb_table, const float* cie,
                          float y_integral, uint64_t jid_begin, uint64_t jid_count, int rng_mode,
                          float* film, float* records);
/* Same, logging every Logger event (worker.cpp:16-48) into events (capacity entries, in job order);
 * *count = events produced. */
int vpto_render_jobs_events(const vpt_configuration* cfg, const vpto_grid* density,
                            const vpto_grid* temperature, const float* bb_table, const float* cie,
                            float y_integral, uint64_t jid_begin, uint64_t jid_count, float* film,
                            vpt_event* events, uint64_t capacity, uint64_t* count);
/* Volume::log_majorant_trace (volume.cpp:176-192): [max_rows][9] rows; returns the segment count. */
/* Volume::log_dda_trace (src/volume.cpp:194-225): rows as vpt_dda_row; returns the voxel count or
 * -1 when the ray misses the index bbox. */
int vpto_dda_trace(const vpto_grid* density, const float* origin3, const float* dir3, vpt_dda_row* rows, int max_rows);
int vpto_majorant_trace(const vpto_grid* density, const float* origin3, const float* dir3, float* rows,
                        int max_rows);

/* The reference worker pool (src/main.cpp:62-87): num_workers threads calling run() over a
 * TileProvider(output_size, num_waves, tile_size).  Returns wall milliseconds (or <0 on error). */
double vpto_render_pool(const vpt_configuration* cfg, const vpto_grid* density,
                        const vpto_grid* temperature, const float* bb_table, const float* cie,
                        float y_integral, uint32_t num_waves, int num_workers, float* film,
                        vpt_counters* counters);

/* Synthetic stand-in grids, generated independently of the product:
 * kind 0: constant density 1.0, index [0,n)^3, world = index - n/2 (C2 with n=128)
 * kind 1: procedural cloud density, index [0,n)^3, world = index - n/2 (C3, n=512)
 * kind 2: procedural temperature 40*base on the same lattice (C4)
 * Leaves whose 512 voxels are all zero are omitted; voxels != 0 are active.
 * Returns an owned desc (free with vpto_synth_free). */
vpt_grid_desc* vpto_synth_grid(int kind, int n);
void vpto_synth_free(vpt_grid_desc* d);

/* film_to_image (src/main.cpp:12-24): film[h][w][4] -> rgb8[h][w][3]. */
void vpto_film_to_image(const float* film, int64_t w, int64_t h, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif
