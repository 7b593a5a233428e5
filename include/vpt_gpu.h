/*
 * vpt_gpu.h — C ABI of the MI355X (gfx950) volumetric path-tracing integrator.
 *
 * This is the drop-in boundary for the reference's per-tile integration loop
 *
 *     void vpt::run(const WorkerParameters&, const Volume&, const Camera&, TileProvider&,
 *                   Image<float,4>& film, RandomNumberGenerator rng)
 *         — reference include/vpt/worker.hpp:11, src/worker.cpp:92-208
 *
 * The reference has no FFI or plugin registry: `run` is a plain C++ function called by
 * `num_workers` std::jthreads (src/main.cpp:63-68).  This header exposes the same work as
 * an opaque-context C API with plain pointers and sizes.  A (tile, wave) job is keyed by
 * its job id `jid` exactly as TileProvider::next() assigns it (src/tile_provider.cpp:27-31):
 *     tile = jid % T,  wave = 1 + jid / T,  T = ceil(W/tw) * ceil(H/th)
 * and its random stream is pcg32_fast seeded with hash(seed, jid) (include/vpt/random.hpp:93-95),
 * so any partition of the jid space (threads, launches, GPUs) renders the same samples.
 *
 * Every function returns VPT_OK (0) or an error code; vpt_last_error() gives the message
 * (thread-local).  The reference's fatal paths (`vptFATAL` = exit(1), include/vpt/logging.hpp:16)
 * become error returns here.
 *
 * INTEGRATION.md shows the reference-side binding (a `run_gpu` with run()'s signature).
 */
#ifndef VPT_GPU_H
#define VPT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VPT_ABI_VERSION 1

enum {
  VPT_OK = 0,
  VPT_E_INVALID = 1,  /* bad argument / schema violation */
  VPT_E_HIP = 2,      /* HIP runtime failure or no HIP device */
  VPT_E_IO = 3,       /* file could not be read */
  VPT_E_PARSE = 4,    /* JSON syntax error, missing or unknown key */
  VPT_E_NOMEM = 5,
  VPT_E_STATE = 6     /* call not valid in the context's current state */
};

/* ---- scene configuration: include/vpt/configuration.hpp:14-65 ------------------------- */

/* CameraParameters, configuration.hpp:20-27 */
typedef struct vpt_camera_params {
  float position[3];
  float look[3];
  float up[3];
  float vfov_deg;
  float imaging_ratio;
} vpt_camera_params;

/* WorkerParameters, configuration.hpp:40-50 (image_point_t = Eigen::Index pair) */
typedef struct vpt_worker_params {
  int32_t single_pixel_enabled;
  int32_t use_jitter;
  int64_t single_pixel_coord[2]; /* (x, y) */
  float infinite_light_xyz[3];
  float infinite_light_multiplier;
  float distant_light_xyz[3];
  float distant_light_multiplier;
  float distant_light_inv_direction[3];
  uint32_t max_depth;
} vpt_worker_params;

/* VolumeParameters, configuration.hpp:52-59 */
typedef struct vpt_volume_params {
  float henyey_greenstein_g;
  float le_scale;
  float sigma_a;
  float sigma_s;
  float temperature_offset;
  float temperature_scale;
} vpt_volume_params;

/* Configuration, configuration.hpp:61-71 */
typedef struct vpt_configuration {
  uint32_t seed;
  uint32_t num_waves;
  uint32_t num_workers;
  uint32_t _pad0;
  int64_t output_size[2]; /* (w, h) */
  int64_t tile_size[2];   /* (w, h) */
  vpt_camera_params camera_parameters;
  vpt_worker_params worker_parameters;
  vpt_volume_params volume_parameters;
  char volume_path[4096]; /* as written in the JSON (relative to the config's directory) */
} vpt_configuration;

/* read_configuration (src/configuration.cpp:8-22): strict JSON reader for exactly this schema;
 * a missing key (glaze error_on_missing_keys) or an unknown key is VPT_E_PARSE. */
int vpt_config_read(const char* path, vpt_configuration* out);
int vpt_config_parse(const char* json_text, size_t len, vpt_configuration* out);

/* ---- grids: include/vpt/volume_grids.hpp:12-14 (nanovdb::NanoGrid<float>) -------------- */

/* A NanoVDB float grid flattened to plain arrays.  Node semantics are NanoVDB's:
 * leaves 8^3, lower nodes 16^3 leaves (128^3 voxels), upper nodes 32^3 lower nodes
 * (4096^3 voxels), root tiles keyed by 4096-aligned origin.  Node existence is implied:
 * a lower node exists if it holds a leaf or a level-1 tile (or is listed in lower_origin),
 * an upper node exists if it holds a lower node or a level-2 tile (or is listed).
 * Slots not covered by a child or a listed tile hold (background, inactive). */
typedef struct vpt_grid_desc {
  float map_mat[9];      /* nanovdb::Map::mMatF    (index->world, row-major) */
  float map_inv_mat[9];  /* nanovdb::Map::mInvMatF (world->index, row-major) */
  float map_vec[3];      /* nanovdb::Map::mVecF    (translation)             */
  float background;
  int32_t index_bbox_min[3]; /* Grid::indexBBox(), inclusive (volume.cpp:83) */
  int32_t index_bbox_max[3];
  uint64_t leaf_count;
  const int32_t* leaf_origin;      /* [leaf_count][3], multiples of 8                      */
  const float* leaf_values;        /* [leaf_count][512], n = (x&7)<<6 | (y&7)<<3 | (z&7)    */
  const uint64_t* leaf_value_mask; /* [leaf_count][8] active-voxel bits (NanoVDB Mask<3>)  */
  const float* leaf_max;           /* [leaf_count] LeafNode::getMax() as stored            */
  uint64_t tile_count;
  const int32_t* tile_origin; /* [tile_count][3]                                                    */
  const int32_t* tile_level;  /* 1: lower-node tile (8^3), 2: upper-node tile (128^3), 3: root tile */
  const float* tile_value;
  const uint8_t* tile_active;
  uint64_t lower_count;       /* optional extra internal nodes that hold no leaf (may be 0)  */
  const int32_t* lower_origin;
  uint64_t upper_count;
  const int32_t* upper_origin;
} vpt_grid_desc;

/* A nanovdb::NanoGrid<float> in memory -> vpt_grid_desc.  grid_buffer = the grid's own bytes, as the
 * reference holds them (&vol.grids().density(), grid.gridSize() bytes = GridHandle::data(); NanoVDB
 * 32.x layout restated, include/vpt/volume_grids.hpp:12-33): leaves with their values, value masks and
 * stored maxima, lower / upper node tiles (non-child slots that are active or differ from the
 * background), root tiles, and every internal node's origin.  Every offset in the buffer is
 * bounds-checked (VPT_E_INVALID on a malformed buffer).  *out owns its arrays: release it with
 * vpt_grid_free.  Replaces the NanoVDB tree walk a caller of vpt_gpu_create would otherwise write. */
int vpt_grid_from_nanovdb(const void* grid_buffer, size_t bytes, vpt_grid_desc** out);
/* nanovdb::io::readGrid(path, grid_name) for a float grid (src/volume_grids.cpp:38-67): .nvdb files
 * of NanoVDB 32.x, codec NONE or ZIP.  A file without a grid of that name returns VPT_OK with
 * *out = NULL (the reference's nanovdb_try_read_grid, volume_grids.cpp:38-46); an unreadable file is
 * VPT_E_IO, a malformed one VPT_E_INVALID.  Release *out with vpt_grid_free. */
int vpt_grid_read_nvdb(const char* path, const char* grid_name, vpt_grid_desc** out);
/* Releases a desc from vpt_grid_from_nanovdb / vpt_grid_read_nvdb / vpt_synth_grid. */
void vpt_grid_free(vpt_grid_desc* desc);

/* fix_majorants_for_interpolation(grid, order=1) (src/volume.cpp:104-160), host side:
 * out_leaf_max[i] = max(desc.leaf_max[i], getValue(c) for c in the 26 neighbour leaf boxes
 * intersected with leaf i's bbox expanded by 1).  Idempotent.  Uses up to num_threads threads. */
int vpt_fix_majorants(const vpt_grid_desc* grid, float* out_leaf_max, int num_threads);

/* ---- blackbody emission: src/precompute_blackbody.cpp:7-52, src/spectral.cpp:7-20 ------- */

#define VPT_BLACKBODY_ROWS 500
/* init_blackbody_radiation_xyz(): bb_xyz[i] = spectrum_to_xyz(planck(T = (i-1)*100 K)),
 * written as [500][3] floats, from the CIE 1931 table shipped with the package. */
int vpt_blackbody_table(float* out_500x3);
/* blackbody_radiation_xyz(T) on the host, for tests. */
int vpt_blackbody_xyz(const float* table_500x3, float temperature_k, float* out_xyz);

/* ---- output: film_to_image (src/main.cpp:12-24, include/vpt/color.hpp:8-30) --------------- */

/* XYZ/W -> linear sRGB (3x3 matrix) -> sRGB OETF -> clamp [0,1] -> *255 -> truncate to u8.
 * film: float[h][w][4]; out: uint8[h][w][3] (the 8-bit RGB image the reference saves as PNG). */
int vpt_film_to_srgb8(const float* film_hxwx4, int64_t w, int64_t h, uint8_t* out_hxwx3);

/* ---- the integrator ---------------------------------------------------------------------- */

typedef struct vpt_gpu_ctx vpt_gpu_ctx;

/* Event counters accumulated by every launch (for algorithmic bytes). */
typedef struct vpt_counters {
  uint64_t samples;        /* film samples written (pixels traced)                     */
  uint64_t dda_steps;      /* HDDA steps taken (volume.cpp:56)                          */
  uint64_t segments;       /* majorant segments returned by RayMajorantIterator::next   */
  uint64_t draws;          /* exponential free-flight draws (sampler.cpp:44)            */
  uint64_t stencils;       /* density trilinear stencil refreshes (cell changes)        */
  uint64_t density_evals;  /* density trilinear evaluations                             */
  uint64_t temp_stencils;  /* temperature trilinear stencil refreshes                   */
  uint64_t scatters;       /* scatter events                                            */
  uint64_t shadow_rays;    /* sample_Ld calls that traced a ray                         */
  uint64_t rng_draws;      /* uniform<float>() calls                                    */
  uint64_t exchanged;      /* paths moved by live-path compaction (vpt_gpu_set_compaction) */
} vpt_counters;

/* Create a context on HIP device `device`.  Copies everything it needs (the grids are
 * flattened into an HBM brick pool + leaf-slot/majorant tables; the caller's arrays may be
 * freed afterwards).  `density` is required (volume_grids.cpp:58-60); `temperature` may be
 * NULL (volume_grids.cpp:61-66).  `blackbody_500x3` may be NULL: the table is then computed
 * with vpt_blackbody_table().  The density grid's leaf maxima are fixed for interpolation
 * here (Volume::Volume, volume.cpp:162-170) — passing already-fixed maxima is harmless.
 * Device memory per grid: 9 KiB per leaf (the stencil pool: per voxel row the 2x2 squares of x = 0..8)
 * plus the cell tables (~12 B per 8^3 cell of the lower nodes' bounding box); the host holds the same
 * while building.  A grid that does not fit the device's free memory is VPT_E_NOMEM before any
 * allocation (e.g. 0.84 GB for the 512^3 cloud stand-in's 90 704 leaves). */
int vpt_gpu_create(const vpt_configuration* cfg, const vpt_grid_desc* density,
                   const vpt_grid_desc* temperature, const float* blackbody_500x3, int device,
                   vpt_gpu_ctx** out);
/* The same context on each of n devices (devices[i]; out[n]) with the grids flattened and majorant-fixed once on
 * the host and uploaded to every device in parallel (the multi-GPU drop-in's setup: one flatten instead of n
 * competing for the host's CPUs).  On failure no context is left (out[] NULL) and vpt_last_error() names the
 * device. */
int vpt_gpu_create_many(const vpt_configuration* cfg, const vpt_grid_desc* density,
                        const vpt_grid_desc* temperature, const float* blackbody_500x3, const int* devices, int n,
                        vpt_gpu_ctx** out);
/* The two halves of vpt_gpu_create_many, for a caller that flattens the grids while the HIP runtime starts
 * (vpt_gpu::run: the flatten is host work and needs no device).  vpt_grids_flatten: the host side of
 * Volume::Volume -- the grids flattened and the density's majorants fixed (no HIP call; the caller's arrays may be
 * freed afterwards).  vpt_gpu_create_from: a context per device from those grids, as vpt_gpu_create_many.  The
 * grids stay the caller's until vpt_grids_free. */
typedef struct vpt_host_grids vpt_host_grids;
int vpt_grids_flatten(const vpt_grid_desc* density, const vpt_grid_desc* temperature, vpt_host_grids** out);
int vpt_gpu_create_from(const vpt_configuration* cfg, const vpt_host_grids* grids, const float* blackbody_500x3,
                        const int* devices, int n, vpt_gpu_ctx** out);
void vpt_grids_free(vpt_host_grids* grids);
int vpt_gpu_destroy(vpt_gpu_ctx* ctx);

/* Jobs per wave T and total jobs num_waves*T of the context's configuration. */
int vpt_gpu_job_space(const vpt_gpu_ctx* ctx, uint64_t* jobs_per_wave, uint64_t* total_jobs);

/* Render jobs [jid_begin, jid_begin + jid_count) asynchronously on `hip_stream`
 * (a hipStream_t; NULL = the null stream, as everywhere in HIP), accumulating into `film_device`:
 * a device float[H][W][4] (X, Y, Z, sample count; image.hpp:40-60) — NULL = the context's own
 * film.  With the ordered film (the default, vpt_gpu_set_film_order) each pixel's samples are
 * added in wave order, the reference's order, so a film rendered from zero equals the reference's
 * bit for bit; with VPT_FILM_ATOMIC they are fp32 atomics in completion order (≈1e-7 relative).
 *
 * Concurrency: launches of one context may be in flight on several streams at once.  Each launch
 * takes its own job counter from a ring of 64 per context; a ring slot is reused only after the
 * launch that last held it has completed (the new launch's stream waits on an event), so any number
 * of launches is safe.  Launches that share a film add into it atomically.  The calls that change
 * context state read by running kernels (vpt_gpu_set_tuning, vpt_gpu_set_rng_mode) and
 * vpt_gpu_film_clear first wait for this context's launches.  One context is driven by one host
 * thread at a time (as the reference's `run` owns its RandomNumberGenerator): a state-changing call
 * made from a second thread while the first is inside vpt_gpu_render_jobs is not supported. */
int vpt_gpu_render_jobs(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count,
                        float* film_device, void* hip_stream);

/* How launches add into the film.  The reference's film receives each pixel's samples in wave order:
 * TileProvider::next() hands a tile's wave out only after its previous wave is released
 * (tile_provider.cpp:40-60), and a job adds each pixel's sample as it is traced (worker.cpp:203-204:
 * w += 1, xyz += imaging_ratio * L).
 *   VPT_FILM_ORDERED (default): a production launch stores every sample's L into a device buffer of
 *     jid_count * tile_w*tile_h * 12 bytes (plain stores, regrouped through the wavefront as the atomics
 *     were), then vpt_film_order_kernel adds them into the film pixel by pixel in wave order: a film
 *     rendered from zero by one launch -- or by launches of consecutive job ranges in jid order -- equals
 *     the reference's bit for bit, and every run gives the same film.  The buffer is the context's (kept
 *     between launches; C3: 6.4 GB, C5 on one GPU: 102 GB); ordered launches of a context run one at a time
 *     (each waits for the previous one's film pass on its stream).  max_bytes caps the buffer (0 = auto:
 *     3/4 of the device's free memory when it grows): a larger launch is split into consecutive launches,
 *     whole waves at a time where the range allows -- the same film.
 *   VPT_FILM_ATOMIC: fp32 atomics as samples complete (the order varies run to run, ≈1e-7 relative).
 * Debug launches (records, events) and feeds always add atomically; so does a launch whose buffer would
 * have to grow while a feed of the context is open.  Growing the buffer frees and allocates device memory,
 * which may wait for the whole device (see the feeds below): with feeds of other contexts open on the same
 * device, size it beforehand (a first ordered launch of the largest range, or max_bytes).  Takes effect at
 * the next launch; VPT_FILM_ATOMIC frees the buffer. */
enum { VPT_FILM_ATOMIC = 0, VPT_FILM_ORDERED = 1 };
int vpt_gpu_set_film_order(vpt_gpu_ctx* ctx, int mode, uint64_t max_bytes);
/* The film mode, the sample buffer's size and the launches that ran ordered / atomic (feeds not counted). */
int vpt_gpu_film_order_info(const vpt_gpu_ctx* ctx, int* mode, uint64_t* buffer_bytes, uint64_t* ordered_launches,
                            uint64_t* atomic_launches);

/* The drop-in's ordered frame (vpt_run.hpp: vpt_gpu::run's film, bit-identical to the reference's).  A feed's jobs
 * arrive in the provider's order and its film is progressive, so its launch adds samples with fp32 atomics; with a
 * frame open, the context's feed launches also store the samples of the jobs of tiles [tile_lo, tile_hi) in waves
 * jid_lo / T .. + *waves - 1 (from job jid_lo on) in the context's sample buffer (*waves * (tile_hi - tile_lo) *
 * tile_area * 12 bytes, allocated here -- before any feed of the context is open: a running feed's launch holds the
 * device, which an allocation may wait for; VPT_E_STATE otherwise).  *waves: asked for in, granted out -- at most
 * what fits 3/4 of the device's free memory and 128 GiB (VPT_E_NOMEM when not one wave does).  After the feeds are collected,
 * vpt_gpu_frame_finish adds the stored samples of jobs [jid_lo, jid_end) pixel by pixel in wave order -- w += 1,
 * xyz += imaging_ratio * L (worker.cpp:203-204) -- onto `prior` (the host film before the frame, float[H][W][4];
 * NULL = zeros) and writes the frame's tiles' pixels into film_host, replacing what the feeds' collects added
 * there.  Every job of those tiles in [jid_lo, jid_end) must have been rendered by this context's feeds (one taker
 * hands out a contiguous range); jid_end beyond the frame's waves is VPT_E_INVALID (those jobs stored nothing).
 * waves = 0 closes the frame; finish closes it too.  While a frame is open the context's other ordered launches add
 * with atomics (the buffer is the frame's). */
int vpt_gpu_frame_open(vpt_gpu_ctx* ctx, uint64_t jid_lo, uint64_t* waves, uint32_t tile_lo, uint32_t tile_hi);
int vpt_gpu_frame_finish(vpt_gpu_ctx* ctx, uint64_t jid_end, const float* prior, float* film_host);

/* Like vpt_gpu_render_jobs but also writes every sample's radiance L (before the
 * imaging_ratio scale) to records_device[(jid - jid_begin) * tile_w*tile_h + y_local*rect_w + x_local][3]
 * — a debug path for bit-exact per-sample parity. */
int vpt_gpu_render_jobs_records(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count,
                                float* film_device, float* records_device, void* hip_stream);

/* ---- debug traces ------------------------------------------------------------ */

/* One line of the reference's event log (Logger<true>, src/worker.cpp:16-48 -> log.csv). */
enum {
  VPT_EV_NEW_RAY = 0,            /* v = camera ray origin xyz, direction xyz (worker.cpp:125)    */
  VPT_EV_SAMPLED_POINT = 1,      /* v = collision point xyz (world), density (worker.cpp:145)    */
  VPT_EV_NULL = 2,               /* (worker.cpp:164)                                             */
  VPT_EV_SCATTER_TERMINATED = 3, /* (worker.cpp:168)                                             */
  VPT_EV_SCATTER = 4,            /* v = new ray origin xyz, direction xyz (worker.cpp:180)       */
  VPT_EV_ABSORBED = 5            /* (worker.cpp:185)                                             */
};
typedef struct vpt_event {
  uint64_t jid;    /* job id                                                    */
  uint32_t pixel;  /* pixel within the job's clipped tile rect, y * width + x   */
  uint32_t seq;    /* order of the event within its job                         */
  uint32_t type;   /* VPT_EV_*                                                   */
  float v[7];
} vpt_event;     /* 48 bytes */

/* Render jobs like vpt_gpu_render_jobs and append every Logger event to events_device (capacity
 * entries, unordered across jobs: sort by (jid, seq)).  *count = events produced (may exceed
 * capacity; the excess is dropped).  Synchronous. */
int vpt_gpu_trace_jobs(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film_device,
                       vpt_event* events_device, uint64_t capacity, uint64_t* count, void* hip_stream);

/* Volume::log_dda_trace (src/volume.cpp:194-225) for one world ray, on the host: the voxels of
 * NanoVDB's unit DDA from 16 index units before to 16 after the ray's clip to the index bbox, with
 * getValue, getDim, getNodeInfo (dim, maximum) and isActive at each (row = one dda_trace.csv line).
 * *n_rows = voxels walked (rows beyond max_rows are not written), or -1 when the ray misses the
 * index bbox (the reference then writes no file). */
typedef struct vpt_dda_row {
  int32_t ijk[3];
  float t;
  float value;
  uint32_t dim_getdim;
  uint32_t dim_nodeinfo;
  int32_t active;
  float maximum;
} vpt_dda_row;
int vpt_dda_trace(const vpt_grid_desc* density, const float origin[3], const float direction[3], vpt_dda_row* rows,
                  int max_rows, int* n_rows);

/* Volume::log_majorant_trace (src/volume.cpp:176-192) for one world ray: per RayMajorantIterator
 * segment the row X0,Y0,Z0,X1,Y1,Z1,T0,T1,Majorant (index-space end points, world-space t).
 * rows_host: [max_rows][9]; *n_rows = segments (0 if the ray misses the volume).  Synchronous. */
int vpt_gpu_majorant_trace(vpt_gpu_ctx* ctx, const float origin[3], const float direction[3],
                           float* rows_host, int max_rows, int* n_rows);

/* Throughput mode.  VPT_RNG_REFERENCE (default): one pcg32_fast stream per job,
 * hash(seed, jid), a job's pixels traced in order -- the reference's samples.  VPT_RNG_PIXEL: every
 * pixel of a job is its own work item with stream hash(seed, jid * tile_area + pixel); it matches
 * the reference only in expectation and is never used for parity. */
enum { VPT_RNG_REFERENCE = 0, VPT_RNG_PIXEL = 1 };
int vpt_gpu_set_rng_mode(vpt_gpu_ctx* ctx, int mode);
/* Throughput mode's work granularity: pixels of one job per work item (a lane traces them in order, each
 * with its own stream, so the samples do not depend on it).  0 (default): the largest power of two
 * dividing the tile area that leaves >= 32 work items per resident lane; else a power of two dividing
 * the tile area (VPT_E_INVALID otherwise).  Applies from the next render call. */
int vpt_gpu_set_pixel_chunk(vpt_gpu_ctx* ctx, int chunk);

/* Kernel variant of density-only scenes.  The run-skipping variant takes, from an interior cell whose
 * majorant equals the segment's, the next r HDDA steps without loading their cells (r = the cell's
 * precomputed run radius); samples are identical.  mode -1 (default): chosen at creation (on when
 * >= 1/4 of the interior cells have r >= 2, e.g. C2's constant cube); 0: off; 1: on (VPT_E_INVALID
 * with a temperature grid).  Takes effect at the next launch. */
int vpt_gpu_set_run_skipping(vpt_gpu_ctx* ctx, int mode);
/* The production kernel the context launches: temperature grid present, run skipping on. */
int vpt_gpu_kernel_variant(const vpt_gpu_ctx* ctx, int* has_temperature, int* run_skipping);

/* Scheduling order of a whole-wave job range (jid_begin and jid_count multiples of T).  Results
 * never depend on it: every job keeps its jid and RNG stream, only the fp32 atomic film-add order
 * changes.  VPT_ORDER_JID: jid order, as TileProvider::next() hands jobs out.
 * VPT_ORDER_COST_WAVE_MAJOR: wave by wave, each wave's tiles costliest first.
 * VPT_ORDER_COST_TILE_MAJOR: the whole range as one costliest-first list -- tiles ranked by cost in
 * groups of 64, each group's waves consecutively (64 lanes = 64 tiles of one wave).
 * VPT_ORDER_COST_TAIL: wave-major, then the last ~6 x (resident lanes / T) waves
 * tile-major, so the launch drains on cheap (sky) jobs without concentrating the whole launch on
 * the densest tiles.
 * VPT_ORDER_COST_SAME_TILE (default): tile by tile, costliest first, each tile's waves consecutively --
 * the 64 lanes of a wavefront take one tile's jobs of 64 waves, so they trace the same pixels and their
 * rays walk the same cells until they scatter; the range drains on the cheapest tiles.  Launches that
 * add with film atomics (the ordered film off, feeds, debug launches) take VPT_ORDER_COST_TAIL instead
 * (64 lanes would add to one pixel at once), and so do partly filled launches (a few jobs per resident
 * lane: C2, a GPU's share of a frame), where it measured slower.  Costs: vpt_gpu_tile_costs.  Other
 * ranges run in jid order. */
enum {
  VPT_ORDER_JID = 0,
  VPT_ORDER_COST_WAVE_MAJOR = 1,
  VPT_ORDER_COST_TILE_MAJOR = 2,
  VPT_ORDER_COST_TAIL = 3,
  VPT_ORDER_COST_SAME_TILE = 4
};
int vpt_gpu_set_job_order(vpt_gpu_ctx* ctx, int mode);
/* VPT_ORDER_COST_TAIL's tile-major wave count (0 = auto: 6 x resident lanes / T, rounded up); also the
 * fallback of VPT_ORDER_COST_SAME_TILE. */
int vpt_gpu_set_job_order_tail(vpt_gpu_ctx* ctx, int waves);
/* The per-tile cost estimates (float[T], may be NULL) and the tile ranks by descending cost
 * (uint32[T], may be NULL): HDDA steps + 4 x majorant optical depth of 5 primary rays per tile. */
int vpt_gpu_tile_costs(vpt_gpu_ctx* ctx, float* cost_T, uint32_t* rank_T);
/* Replaces the cost estimates with caller-supplied per-tile costs (float[T], e.g. measured job times
 * of an earlier launch) and re-ranks the tiles; waits for all work on the device first. */
int vpt_gpu_set_tile_costs(vpt_gpu_ctx* ctx, const float* cost_T);
/* An explicit job order for launches of exactly n jobs (any jid_begin): work item k renders job
 * jid_begin + perm[k].  perm must be a permutation of 0..n-1; n = 0 clears it.  Samples never depend
 * on the order.  Not used in the pixel RNG mode. */
int vpt_gpu_set_job_permutation(vpt_gpu_ctx* ctx, const uint32_t* perm, uint64_t n);

int vpt_gpu_sync(vpt_gpu_ctx* ctx);

/* ---- pipelining and progressive films (the drop-in's drain, include/vpt_run.hpp) ------------ */

/* A HIP stream on the context's device (non-blocking w.r.t. the null stream), for launches that overlap:
 * a launch lasts as long as its longest job (a tile's pixels in one RNG stream), so back-to-back launches
 * on one stream would each pay that drain; launches on two streams fill it with the next one's jobs. */
int vpt_gpu_stream_create(vpt_gpu_ctx* ctx, void** hip_stream);
int vpt_gpu_stream_destroy(vpt_gpu_ctx* ctx, void* hip_stream);
/* Waits for the work enqueued on hip_stream so far. */
int vpt_gpu_stream_sync(vpt_gpu_ctx* ctx, void* hip_stream);
/* Binds the calling thread to the CPUs of the NUMA node the context's device is attached to (intersected
 * with the process's CPU set -- its main thread's, which taskset / numactl restrict -- rather than the
 * calling thread's own, which it inherited from whichever thread created it; *node = that node, or -1 when
 * it is unknown or the intersection is empty, and the thread is left as it was).  A feed's pusher reads and writes the pinned ring, which sits
 * in that node's memory, a slot per job: from the other socket of a 2-socket host every access crosses the
 * socket link (C4 through the drop-in: 174-205 ms per frame with the process on the far node, 119-148 on the
 * GPU's, profiles/archive/r05m_numa.txt).  `node` may be NULL. */
int vpt_gpu_bind_thread_near(vpt_gpu_ctx* ctx, int* node);
/* An extra device film (float[H][W][4], zeroed) of the context's size, e.g. the second buffer of a
 * progressive film; release it with vpt_gpu_film_free before vpt_gpu_destroy. */
int vpt_gpu_film_alloc(vpt_gpu_ctx* ctx, float** film_device);
int vpt_gpu_film_free(vpt_gpu_ctx* ctx, float* film_device);
/* film_host[i] += film_device[i], then film_device = 0 (film_device NULL = the context's own film).
 * Synchronous.  The caller must have waited for every launch that renders into film_device (this call
 * does not know their streams); launches into other films may keep running.  Uses a pinned staging
 * buffer owned by the context. */
int vpt_gpu_film_flush_to_host(vpt_gpu_ctx* ctx, float* film_device, float* film_host_hxwx4);

/* Feeds: one launch of the production kernel that renders job ids pushed by the host while it runs --
 * the drop-in's way of handing the GPU a TileProvider's tokens as they are taken, with a bounded queue and
 * no per-batch launch drain (a launch lasts as long as its longest job; a feed's lanes keep taking pushed
 * jobs instead).  vpt_gpu_feed_open prepares it on hip_stream (a stream of this context,
 * vpt_gpu_stream_create) into film_device (NULL = the context's own film); it is launched once as many jobs
 * are pushed as it has lanes (C3: 458 752), when the window fills, or at close.  `window` (rounded up to a
 * power of two, >= 1024 and >= twice the lanes) bounds the jobs pushed and not yet started:
 * vpt_gpu_feed_push blocks while the window is full (VPT_E_STATE if the launch stops taking jobs for 120 s).  Job ids are any jids (< 2^62), e.g.
 * token.jid(); their samples equal vpt_gpu_render_jobs's.  vpt_gpu_feed_close publishes the end: the
 * launch ends once every pushed job is rendered, then adds their sample counts to the film (asynchronous,
 * on the feed's stream).  vpt_gpu_feed_query: whether a closed feed's work is complete (non-blocking) and
 * the jobs pushed.  vpt_gpu_feed_destroy closes if needed, waits for the feed's work and frees it;
 * VPT_E_STATE if lanes gave up waiting for jobs (a lane waits at most 30 s, so a launch always ends: a
 * feed left open without pushes that long ends by itself).  A feed's launch holds the device's CUs until it
 * is closed -- a second feed opened meanwhile starts as the first one's lanes leave -- so push to a feed
 * only after the feeds opened before it have been closed; and a call that waits for the whole device
 * (hipDeviceSynchronize, and hipFree / hipHostMalloc / hipHostFree may) waits for an open feed's lanes to
 * give up: wait for streams instead.  The context's own calls that wait for its launches (vpt_gpu_sync,
 * vpt_gpu_film_clear, vpt_gpu_film_add_to_host, vpt_gpu_counters, vpt_gpu_profile, vpt_gpu_set_tuning,
 * vpt_gpu_set_latency_tuning, vpt_gpu_set_rng_mode, vpt_gpu_set_tile_costs, vpt_gpu_set_job_permutation,
 * and vpt_gpu_tile_costs before its first cost pass) return VPT_E_STATE while a feed of the context is
 * launched and not closed, instead of waiting 30 s for its lanes to give up.  A destroyed feed's memory is
 * kept by the context for the next vpt_gpu_feed_open (freed by vpt_gpu_destroy).  Feeds use a host-pinned
 * ring (8 bytes per window slot) and run the reference RNG mode. */
typedef struct vpt_gpu_feed vpt_gpu_feed;
int vpt_gpu_feed_open(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window, vpt_gpu_feed** out);
int vpt_gpu_feed_push(vpt_gpu_feed* feed, const uint64_t* jids, uint64_t n);
int vpt_gpu_feed_close(vpt_gpu_feed* feed);
int vpt_gpu_feed_query(vpt_gpu_feed* feed, int* done, uint64_t* pushed);
int vpt_gpu_feed_destroy(vpt_gpu_feed* feed);
/* Jobs pushed and not yet taken by a lane -- an estimate: the lanes report every 1 024th job they take into
 * 4 words of the pinned block (their posted writes land in any order; the largest counts); before the launch
 * every pushed job counts.  It can read high, never for long while the lanes wait: a wavefront that finds
 * every published job taken stores the job count it saw (again every ~5 ms while it waits), and a count >= the
 * published one reads as 0; hints that have not moved for 10 ms read as 0 too.
 * Cheap: a read of one cache line. */
int vpt_gpu_feed_backlog(vpt_gpu_feed* feed, uint64_t* backlog);
/* Test hook for the backlog estimate's words (tests/test_gpu_integration.py): op 0 reads the "waiting" word into
 * *value, op 1 writes *value into it, op 2 writes *value into every reservation hint (and the host's view of
 * them) -- a stale value landing last, which waiting wavefronts overwrite within ~5 ms (they store the count they
 * see every 2^19 ticks of s_memrealtime) and the estimate ignores after 10 ms without a new hint. */
int vpt_gpu_feed_debug(vpt_gpu_feed* feed, int op, uint64_t* value);
/* A staged feed renders into film_device (NULL = the context's own film), which must be zero, on hip_stream
 * (NULL = a stream of the feed's own), and counts the jobs it completes per tile; its film reaches the host through the copy engines, which run beside a launch
 * that holds every CU (r05), so nothing in its life waits for CUs another feed's launch holds.
 *   vpt_gpu_feed_snapshot -- at any time, also while the launch runs: adds into film_host (film_count
 *     floats, the reference's [H][W][4] layout) what the launch has rendered since the previous snapshot --
 *     the completed jobs' sample counts and the film's radiance as copied (~2 ms for a 1080p film).  A
 *     progressive film (main.cpp:101-132's 5-FPS window): every snapshot's additions telescope to the final
 *     film (to fp32 rounding, see collect).  The caller serialises writers of film_host.
 *   vpt_gpu_feed_collect -- closes if needed, waits for the launch, adds the rest, clears film_device and
 *     frees the feed like destroy.  The sample counts then end exact (whole jobs per tile); the radiance ends
 *     equal to the launch's film within fp32 rounding (each snapshot adds a rounded difference, and several
 *     drivers may share film_host).  An intermediate snapshot's radiance includes samples of jobs still
 *     running while their counts arrive only when each job ends, so a progressive frame reads slightly bright
 *     until its jobs complete.
 * vpt_gpu_feed_prepare allocates a feed's memory (the ring, and with staged != 0 the copy buffers) into the
 * context's pool ahead of the first open, e.g. right after vpt_gpu_create, so that no allocation runs while a
 * launch holds the device. */
int vpt_gpu_feed_open_staged(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window,
                             vpt_gpu_feed** out);
int vpt_gpu_feed_snapshot(vpt_gpu_feed* feed, float* film_host);
int vpt_gpu_feed_collect(vpt_gpu_feed* feed, float* film_host);
int vpt_gpu_feed_prepare(vpt_gpu_ctx* ctx, uint64_t window, int staged);

/* Zero the context's own film. */
int vpt_gpu_film_clear(vpt_gpu_ctx* ctx);
/* Device pointer of the context's own film (for an RCCL reduce), and its element count H*W*4. */
int vpt_gpu_film_device_ptr(vpt_gpu_ctx* ctx, float** film_device, uint64_t* count);
/* film_host[i] += own film[i] (synchronous), the caller-owned reference-layout film. */
int vpt_gpu_film_add_to_host(vpt_gpu_ctx* ctx, float* film_host_hxwx4);
/* Counters summed over every launch since creation (or the last reset). */
int vpt_gpu_counters(vpt_gpu_ctx* ctx, vpt_counters* out, int reset);
/* Scheduling knobs (results never depend on them): a rare lane state (new job, new pixel, ray
 * setup, NEE completion, film write) runs when >= gate_min lanes of a wavefront wait for it or
 * fewer than gate_idle lanes are walking rays; a tentative collision's density evaluation waits
 * for gate_eval lanes likewise; grid_blocks overrides the persistent grid size; the ray walk
 * repeats in an inner loop while >= gate_walk lanes walk (0: one step per pass).
 * Pass <= 0 (gate_idle, gate_walk < 0) to keep a value; gate_idle 0 is rejected (VPT_E_INVALID): a
 * wavefront with no walking lane must run its waiting blocks. */
int vpt_gpu_set_tuning(vpt_gpu_ctx* ctx, int gate_min, int gate_idle, int grid_blocks, int gate_eval,
                       int gate_walk);
/* Latency-bound launches: a launch with fewer work items than its grid has lanes (e.g. C1, 4 096
 * jobs) lasts as long as its slowest job.  Such launches spread their items over the grid's
 * wavefronts -- the first wave_lanes lanes of each wavefront take jobs (0 = auto: 1 while items /
 * wavefronts < 3, each lane taking its jobs in sequence, else 1 + floor(items / wavefronts)) -- and run with their own gates (meaning as in vpt_gpu_set_tuning; defaults 1, 65, 1, 1:
 * every block runs as soon as one lane needs it).  Results never depend on them.  Pass < 0 (gate_min,
 * gate_eval: <= 0) to keep a value; gate_idle 0 is rejected. */
int vpt_gpu_set_latency_tuning(vpt_gpu_ctx* ctx, int wave_lanes, int gate_min, int gate_idle, int gate_eval,
                               int gate_walk);
/* The latency kernel: the same state machine with the lane's cold state in VGPRs instead of LDS and a
 * larger register budget (4-5 waves per SIMD instead of 7), for launches that occupy at most that many
 * anyway.  mode -1 (default): latency-bound launches (C1: 20.7-21.2 -> 19.2-19.7 ms) and partly filled ones
 * whose grid rule gives <= its resident blocks per CU (C2: 100-101 -> 95.7-96.6 ms; a GPU's small share of a
 * frame); 0: never; 1: always (tests, A/B).  ungated 0 (default): partly filled launches on it use the
 * context's gates; 1: the latency gates (every block runs for one waiting lane, vpt_gpu_set_latency_tuning;
 * measured slower there: C2 109 ms); -1: keep.  Latency-bound launches always use the latency gates.
 * Samples never depend on it.  Takes effect at the next launch. */
int vpt_gpu_set_latency_kernel(vpt_gpu_ctx* ctx, int mode, int ungated);
/* Live-path compaction (north_star's "ballot/prefix-sum to compact live rays") on the latency kernel's partly
 * filled launches (e.g. C2): every `every` outer iterations a block's four wavefronts meet and, when packing
 * helps, move their paths through LDS so that walking paths fill the first wavefronts (a kernel variant with a
 * 60 KiB LDS exchange: <= 2 blocks per CU; launches with more blocks per CU do not use it).  0 (default): off.
 * Samples never depend on it (counters: `exchanged`).  Takes effect at the next launch. */
int vpt_gpu_set_compaction(vpt_gpu_ctx* ctx, int every);
/* The mode and the latency kernel's resident blocks per CU. */
int vpt_gpu_latency_kernel_info(const vpt_gpu_ctx* ctx, int* mode, int* resident_blocks_per_cu);
/* SIMT-utilisation profile of profiling builds (-DVPT_PROFILE): for each block of the lane state
 * machine, [wave executions, active lanes] as 2*21 uint64 (the last 7: lanes per state at each walk-loop iteration), then the shader cycles the wavefronts
 * spent in each of 10 sections (fetch, pixel, ray, walk-loop control, eval, nee, finish, and the
 * walk's segment / step / draw parts); zeros in normal builds.  n must be >= 2 * 21 + 10. */
int vpt_gpu_profile(vpt_gpu_ctx* ctx, uint64_t* out, int n, int reset);
/* Launch geometry used by the integrator kernel (for reports). */
int vpt_gpu_launch_info(const vpt_gpu_ctx* ctx, int* grid_blocks, int* block_threads);
/* Number of HIP devices (0 without a GPU: VPT_OK, *count = 0). */
int vpt_gpu_device_count(int* count);
/* The drop-in's seed recovery on the GPU: the u32 seeds s (ascending, at most max_seeds written) whose job-0
 * stream -- pcg32_fast seeded with hash(s, 0) (hash.hpp:20-67, random.hpp:93-95) -- starts with the outputs
 * out0, out1; *n_found = how many exist (normally 1).  The reference's RandomNumberGenerator keeps its seed
 * private (random.hpp:86-115), so include/vpt_run.hpp finds it from two draws: all 2^32 candidates in one
 * launch on `device` (a few ms; the same scan took 1-3 s on 8-16 host threads).  Synchronous. */
int vpt_gpu_find_seeds(int device, uint32_t out0, uint32_t out1, uint32_t* seeds, int max_seeds, int* n_found);
/* What vpt_gpu_create and the first cost pass took (ms), n <= 5 of: [0] grid flatten + leaf-majorant fix (host),
 * [1] grid upload, [2] the rest of the context (tables, buffers, occupancy, scene constants), [3] the tile-cost
 * pass (vpt_gpu_tile_costs / the first cost-ordered launch), [4] binding the device (hipSetDevice: the HIP
 * runtime's start when it is the process's first HIP call). */
int vpt_gpu_setup_timings(const vpt_gpu_ctx* ctx, double* ms, int n);

/* ---- synthetic stand-in volumes (the reference's .nvdb files are not available) ---------- */

/* kind 0: constant density 1.0 over index [0,n)^3 (n = 128)
 * kind 1: procedural cloud density over [0,n)^3 (C3, n = 512):
 *         p = (ijk + 0.5)/(n/2) - 1, base = clamp((0.85 - |p|)/0.35, 0, 1),
 *         density = base * (0.5 + 0.5 sin(11px+2) sin(13py+1) sin(17pz+3))  (double, then float)
 * kind 2: temperature 40*base on the same lattice (C4)
 * world = index - n/2; leaves with no non-zero voxel are omitted; non-zero voxels are active;
 * indexBBox = bbox of active voxels; leaf_max = max over active voxels.  NULL on bad arguments.
 * The returned desc owns its arrays: release it with vpt_synth_free. */
vpt_grid_desc* vpt_synth_grid(int kind, int n);
void vpt_synth_free(vpt_grid_desc* desc);

/* Thread-local message for the last non-OK return. */
const char* vpt_last_error(void);
int vpt_abi_version(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* VPT_GPU_H */
