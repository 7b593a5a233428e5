// vpt_kernels.h — the integrator's device code: the launch arguments, the kernel environment (cold lane
// state in LDS or VGPRs, the feed protocol's fetch, the regrouped film adds / ordered-film stores), live-path
// compaction, and the kernels (integrator, film passes, seed search, majorant trace, tile costs).  Included by
// vpt_gpu.hip only (the translation unit that launches them).
#pragma once

#include <hip/hip_runtime.h>

#include "vpt_internal.h"
#include "vpt_launch.h"

namespace vpt {

constexpr int kCounterCount = CNT_COUNT;
// Minimum waves per SIMD (launch bounds): 7 for the production density-only kernel (72 VGPRs; the
// cold lane state lives in LDS, see LaneCold), 6 for the temperature kernel (C4: 3748 Msps at its
// natural 5, 3809 at 6, 3684 at 7), 4 for the per-sample-record / event variants.  The kernel is latency-bound enough that occupancy pays: persistent grids of 3/4/5
// blocks per CU measured 802/956/1067 Msps on C3 with one binary; 6 waves 1155, 7 waves 1194.
#ifndef VPT_WAVES_FAST
#define VPT_WAVES_FAST 7
#endif
#ifndef VPT_WAVES_SLOW
#define VPT_WAVES_SLOW 4
#endif
#ifndef VPT_WAVES_TEMP
#define VPT_WAVES_TEMP 6
#endif
// The latency kernel (partly filled and latency-bound launches: C1, C2, a GPU's small share of a frame):
// at most VPT_WAVES_LAT waves per SIMD run anyway there, so it trades occupancy for registers -- the
// lane's cold state in VGPRs instead of LDS (no LDS round trips on the per-pixel / per-bounce chain)
// and a 512 / VPT_WAVES_LAT register budget.
#ifndef VPT_WAVES_LAT
#define VPT_WAVES_LAT 4
#endif

// The lanes' cold state (vpt_integrator.h LaneCold), one slot per thread of the integrator's block.
__shared__ LaneCold g_lane_cold[kBlockThreads];
// LDS copies of the small lookup tables the evaluation reads per lane (logf's 16 x 2 doubles; the
// temperature kernel's 501 x 3 blackbody table): LDS reads instead of vector-memory loads, which
// would count in vmcnt with the walk's loads.
__shared__ double g_logf_tab[16][2];
constexpr int kBbFloats = kBbLdsRows * 3;


// A launch's arguments (the host fills them; the integrator kernel's first argument).
struct KernelArgs {
  uint64_t jid_begin;
  uint64_t jid_count;
  unsigned long long* job_counter;
  float* film;
  float* records;
  int32_t tile_area;
  uint32_t pixel_chunk;  // throughput mode: pixels per work item (a power of two dividing tile_area; else 1)
  unsigned long long* prof_buf;  // [PB_COUNT][2] wave executions, active lanes; then [PT_COUNT] cycles
  const uint32_t* order;             // job order: tile ranks (nullptr = jid order), see ordered_job
  const uint32_t* perm;              // explicit job order (item k -> job perm[k]), overrides order
  uint32_t order_tail_k0;
  uint32_t order_tail_n;
  uint32_t order_group;               // tiles per group of the tile-major part (64; 1: same-tile order)
  vpt_event* events;                 // Logger events (trace launches only)
  unsigned long long* event_count;
  uint64_t event_cap;
  // Feed mode (vpt_gpu_feed_*: the launch takes job ids the host pushes while it runs): host-pinned
  // coherent memory shared with the host -- the published word (items published | kFeedClosed), the
  // ring of job ids (kFeedEmpty once read), the error word and the started hint.  nullptr: items are
  // job_counter values < jid_count (every other launch).
  const uint64_t* feed_word;
  uint64_t* feed_ring;
  uint64_t feed_mask;                // ring slots - 1 (a power of two)
  unsigned* feed_error;
  uint64_t* feed_started;            // [kHintSlots]: a lane that reserves item k, k % kStartedHint == 0, stores k
  uint64_t* feed_waiting;            // a wavefront whose lanes find every published item taken stores the count
  uint32_t feed_hint_mask;           // hint slots - 1
  uint32_t* tile_done;               // a staged feed: jobs completed per tile (device memory), else nullptr
  uint32_t compact_every;            // the compacting latency kernel: outer iterations between two meetings
  // The ordered film (vpt_gpu_set_film_order): every sample's L, plain stores, at
  // samples[(j * tile_area + local pixel) * 3 + c] (j = the job's index in the launch, the records layout);
  // vpt_film_order_kernel then adds them into the film pixel by pixel in wave order.  nullptr: film atomics.
  float* samples;
  // The drop-in's ordered frame (vpt_gpu_frame_open; feed launches only): the samples of job jid = w * T + t of the
  // frame's tiles [frame_tile_lo, frame_tile_lo + frame_tiles) are also stored at frame + (slot * tile_area + local
  // pixel) * 3, slot = (w - frame_w0) * frame_tiles + t - frame_tile_lo (< frame_slots, else not stored), and
  // vpt_frame_order_kernel later adds them into the film in wave order.  nullptr: no frame (the film's atomics alone).
  float* frame;
  uint64_t frame_w0;
  uint64_t frame_slots;
  uint32_t frame_tile_lo;
  uint32_t frame_tiles;
};
typedef const __attribute__((address_space(4))) KernelArgs* ArgsPtr;
// This workgroup's event counters and (VPT_PROFILE builds) section cycles; the temperature kernel's LDS copy of
// S.bb's first kBbLdsRows rows.
__shared__ unsigned long long g_wg_counters[kCounterCount];
#if defined(VPT_PROFILE) || defined(VPT_PROFILE_TIME)
__shared__ unsigned long long g_wg_prof[PT_COUNT + kBlockThreads / 64];
#endif
__shared__ float g_bb_lds[kBbFloats];
// A finish-block pass's samples, per wavefront by rank: (pixel index << 6) | lane (KernelEnvT::film_add / film_commit).
__shared__ uint32_t g_film_rank[kBlockThreads];

// The kernel's view of its launch.  RegCold: the latency kernel's (the lane's cold state in VGPRs).  Feed: a feed
// launch's (job ids from the host's ring, fetch_feed); other launches compile the feed protocol out.  The
// arguments are read where they are used, through an opaque pointer to the kernel's argument segment (scalar
// loads, as the scene's constants are, see ScenePtr): loads the optimiser cannot hoist, so no argument stays live
// in SGPRs across the state-machine loop (they spilled to VGPR lanes: v_readlane / v_writelane in every block).
template <bool RegCold, bool Feed = false>
struct KernelEnvT {
  static_assert(!(RegCold && Feed), "feeds run the throughput kernels only");
  __device__ __forceinline__ ArgsPtr args() const {
    ArgsPtr p = (ArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();  // (KernelArgs is the first argument: offset 0)
    asm volatile("" : "+s"(p));
    return p;
  }

  // Adds w for every active lane with w != 0 (w uniform per call site) to a workgroup counter.
  __device__ __forceinline__ void tally(int32_t k, int32_t w) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(w != 0);
    if (m && __lane_id() == (uint32_t)__builtin_ctzll(m))
      atomicAdd(g_wg_counters + k, (unsigned long long)(__popcll(m) * (uint64_t)(w ? w : 1)));
  }

  __device__ __forceinline__ void prof(int32_t id) {
#ifdef VPT_PROFILE
    const unsigned long long m = __ballot(1);
    if ((__lane_id() == (uint32_t)__builtin_ctzll(m))) {
      atomicAdd(args()->prof_buf + 2 * id, 1ULL);
      atomicAdd(args()->prof_buf + 2 * id + 1, (unsigned long long)__popcll(m));
    }
#else
    (void)id;
#endif
  }
  // Adds n (wave-uniform) to slot id's lane total and 1 to its executions (VPT_PROFILE).
  __device__ __forceinline__ void prof_add(int32_t id, int32_t n) {
#ifdef VPT_PROFILE
    const unsigned long long m = __ballot(1);
    if ((__lane_id() == (uint32_t)__builtin_ctzll(m))) {
      atomicAdd(args()->prof_buf + 2 * id, 1ULL);
      atomicAdd(args()->prof_buf + 2 * id + 1, (unsigned long long)n);
    }
#else
    (void)id;
    (void)n;
#endif
  }
  // Wave time since the previous tick, charged to section id (first active lane; VPT_PROFILE).
  __device__ __forceinline__ void tick(int32_t id) {
#if defined(VPT_PROFILE) || defined(VPT_PROFILE_TIME)
    // the previous tick's time lives in LDS per wavefront (ticks may run under partial masks)
    const unsigned long long t = clock64();
    const unsigned long long m = __ballot(1);
    if (__lane_id() == (uint32_t)__builtin_ctzll(m)) {
      unsigned long long* last = g_wg_prof + PT_COUNT + threadIdx.x / 64;
      atomicAdd(g_wg_prof + id, t - *last);
      *last = t;
    }
#else
    (void)id;
#endif
  }
  // One Logger line (src/worker.cpp:16-48); a = xyz, b = xyz or (b == nullptr) x in v[3].
  __device__ __forceinline__ void event(Lane& ln, uint32_t type, const float* a, const float* b, float x) {
    vpt_event* const events = args()->events;
    if (!events) return;
    const unsigned long long slot = atomicAdd(args()->event_count, 1ULL);
    const uint32_t seq = ln.n_events++;
    if (slot >= args()->event_cap) return;
    vpt_event* e = events + slot;
    e->jid = args()->jid_begin + ln.jid_local;
    e->pixel = (uint32_t)((cold().pix & kPixelMask) - 1);
    e->seq = seq;
    e->type = type;
    for (int i = 0; i < 3; ++i) {
      e->v[i] = a ? a[i] : 0.0f;
      e->v[3 + i] = b ? b[i] : (i == 0 ? x : 0.0f);
    }
    e->v[6] = 0.0f;
  }
  // The lane's cold state: its LDS slot, or (RegCold, the latency kernel) a kernel local the compiler
  // keeps in VGPRs.
  LaneCold* reg_cold;
  __device__ __forceinline__ LaneCold& cold() {
    if constexpr (RegCold)
      return *reg_cold;
    else
      return g_lane_cold[threadIdx.x];
  }
  __device__ __forceinline__ const double (*logf_table() const)[2] { return g_logf_tab; }
  // blackbody_radiation_xyz from the LDS rows when the grid's temperatures stay in them (a uniform
  // branch, so each path keeps its own address space: ds_read or global loads, no flat pointer)
  __device__ __forceinline__ void blackbody(const DevScene& S, float t, float& X, float& Y, float& Z) const {
    if (S.bb_lds_ok)
      blackbody_xyz(S, g_bb_lds, t, X, Y, Z);
    else
      blackbody_xyz(S, S.bb, t, X, Y, Z);
  }
#ifdef VPT_JOB_LOG
  // diagnostic build: per job (tile, fetch time, end time, hardware id) into the records buffer
  __device__ __forceinline__ void job_done(uint32_t job, uint32_t tile, uint32_t t0) {
    uint32_t* e = reinterpret_cast<uint32_t*>(args()->records) + 4 * (uint64_t)job;
    e[0] = tile;
    e[1] = t0;
    e[2] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    e[3] = (blockIdx.x << 8) | threadIdx.x;
  }
#endif
  // lanes of this wavefront for which pred holds
  // (ballot_w64 on the bool itself: the compare folds into the mask, no materialised 0/1 VGPR)
  __device__ __forceinline__ int32_t count(bool pred) { return (int32_t)__popcll(__builtin_amdgcn_ballot_w64(pred)); }
  // wave_lanes: the lanes of each wavefront that take jobs (64: all; fewer in latency-bound launches,
  // see render()); the others end at their first fetch.  Any value >= 1 renders every job: a lane
  // takes jobs until none is left.  0 = auto from x = items / wavefronts: one lane (its jobs in
  // sequence) while x < 3, else 1 + floor(x).  A second path in a wavefront slows the first ~1.6x, so
  // one lane with a few jobs in a row wins: C1 frames on the full grid (r02g,
  // profiles/archive/r02g_c1_lanes_sweep.txt), 1 / 2 / 3 lanes: 8 spp (x = 1.1) 23.3 / 29.3 / - ms, 16 spp
  // (x = 2.3) 31.7 / 32.5 / 35.6, 32 spp (x = 4.6) 51.9 / 43.1 / 42.1 (5 lanes: 41.5).
  // Feed mode: a fetching lane of this wavefront holds a reserved item it has not read (it pins a ring slot
  // until it does), so the fetch block runs now rather than when enough lanes wait (see fetch_feed).
  __device__ __forceinline__ bool fetch_urgent(bool fetching) {
    if constexpr (Feed)
      return count(fetching && cold().pix == kFeedPending) > 0;
    else
      return false;
  }
  __device__ __forceinline__ int fetch_job(uint64_t& j, int32_t wave_lanes) {
    if constexpr (Feed) return fetch_feed(j);
    if (wave_lanes == 0) {
      const float x = (float)args()->jid_count * __builtin_amdgcn_rcpf((float)(gridDim.x * (kBlockThreads / 64)));
      wave_lanes = x < 3.0f ? 1 : 1 + (int32_t)x;
    }
    if ((int32_t)__lane_id() >= wave_lanes) return false;
    unsigned long long v = atomicAdd(args()->job_counter, 1ULL);
    if (v >= args()->jid_count) return 0;
    j = v;
    return 1;
  }
  // Feed mode: the lane reserves item k (one atomic on the launch's counter) and keeps it in its cold
  // state (item_lo / item_hi; pix = kFeedPending) until the host has published it: then it reads the job
  // id from ring slot k & feed_mask and marks the slot empty for the host to reuse.  A lane reserves only
  // while the counter is below the published count (else it waits with nothing reserved, pix =
  // kFeedWait): a reserved, unpublished item pins its ring slot until its lane asks again, which behind
  // busy wave-mates (the fetch block is gated) can take milliseconds -- and the host's window stalls on
  // that slot (r04 fd: 1.35 s stalls, C3 frame 3.7 s).  Once the feed is closed, items beyond the
  // published count are never published: the lane ends.  A lane that waits kFeedDeadline without either
  // (a host that died) ends too and flags feed_error, so the grid always drains.  The loads and stores of
  // host memory are vector-memory atomics of system scope.
  __device__ int fetch_feed(uint64_t& j) {
    LaneCold& lc = cold();
    const ArgsPtr A = args();
    unsigned long long* const job_counter = A->job_counter;
    const uint64_t* const feed_word = A->feed_word;
    unsigned* const feed_error = A->feed_error;
    const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime();  // 100 MHz
    // System-scope loads of host memory go to the host every time.  The host writes a slot before the word
    // that publishes it (release); the slot is read after an acquire fence that follows the word's load.
    const uint64_t w = __hip_atomic_load(feed_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t published = w & ~kFeedClosed;
    if (lc.pix != kFeedPending) {
      const uint64_t c = __hip_atomic_load(job_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (c >= published) {
        if (w & kFeedClosed) return 0;
        // The lanes have taken every item published: say so (one lane per wavefront, as it starts waiting, and
        // again every kWaitingRefresh ticks while it waits -- lc.y0, free while the lane has no job, holds the
        // last store's time).  The host's backlog estimate comes from hints that may land out of order; a count
        // >= its published count here means the lanes wait for it, whatever the hints say
        // (vpt_gpu_feed_backlog).  The refresh overwrites a stale count that landed last.
        bool say;
        if (lc.pix != kFeedWait) {
          lc.pix = kFeedWait;
          lc.x0 = (int32_t)now;  // wait start
          say = true;
        } else if (now - (uint32_t)lc.x0 > kFeedDeadline) {
          __hip_atomic_store(feed_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // (host memory: a store)
          return 0;
        } else {
          say = now - (uint32_t)lc.y0 > kWaitingRefresh;
        }
        if (say) lc.y0 = (int32_t)now;
        const uint64_t m = __builtin_amdgcn_ballot_w64(say);
        if (m && A->feed_waiting && __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == (uint32_t)__builtin_ctzll(m))
          __hip_atomic_store(A->feed_waiting, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return -1;
      }
      const uint64_t k = atomicAdd(job_counter, 1ULL);
      // the host's backlog estimate (vpt_gpu_feed_backlog): a posted write every kStartedHint items
      if ((k & (kStartedHint - 1)) == 0)
        __hip_atomic_store(A->feed_started + ((k / kStartedHint) & A->feed_hint_mask), k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      lc.item_lo = (uint32_t)k;
      lc.item_hi = (uint32_t)(k >> 32);
      if (lc.pix != kFeedWait) lc.x0 = (int32_t)now;  // wait start
      lc.pix = kFeedPending;
    }
    const uint64_t k = ((uint64_t)lc.item_hi << 32) | lc.item_lo;
    if (k < published) {
      uint64_t* slot = A->feed_ring + (k & A->feed_mask);
      // Acquire after the word's load: the slot's load cannot be satisfied before it (ADVICE / VERDICT r04).
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      j = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // And by construction: a slot holds kFeedEmpty from the lane's mark until the host's next id, and the
      // host writes that id only after it has seen the mark, so a slot read too early can only return
      // kFeedEmpty -- never another job's id.  Such a lane keeps its item and asks again.
      if (j == kFeedEmpty) return -1;
      // The empty mark is stored only once the id has arrived (a posted write may overtake a read on the
      // host link, and the host reuses the slot as soon as it sees the mark): the asm takes j as an input,
      // so the compiler waits for the load before it.
      uint64_t empty = kFeedEmpty;
      asm volatile("" : "+v"(empty) : "v"(j));
      __hip_atomic_store(slot, empty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      lc.pix = 0;
      return 1;
    }
    if (w & kFeedClosed) return 0;
    if (now - (uint32_t)lc.x0 > kFeedDeadline) {
      __hip_atomic_store(feed_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // (host memory: a store)
      return 0;
    }
    return -1;
  }
  // A job starts (its id jid): with an ordered frame, a feed lane keeps the address of the job's samples in its cold
  // state (item_lo / item_hi: free once the job is read).  Other launches: nothing.
  __device__ __forceinline__ void job_start(const DevScene& S, LaneCold& lc, uint64_t jid) {
    if constexpr (Feed) {
      if (float* const frame = args()->frame) {
        const uint64_t w = jid / S.T;
        const uint32_t tt = (uint32_t)(jid - w * S.T) - args()->frame_tile_lo;  // (wraps below the band: > tiles)
        const uint64_t slot = (w - args()->frame_w0) * args()->frame_tiles + tt;
        const bool in = tt < args()->frame_tiles && w >= args()->frame_w0 && slot < args()->frame_slots;
        const uint64_t a = in ? (uint64_t)(frame + slot * (uint64_t)S.tile_area * 3) : 0;
        lc.item_lo = (uint32_t)a;
        lc.item_hi = (uint32_t)(a >> 32);
      }
    } else {
      (void)S;
      (void)lc;
      (void)jid;
    }
  }
  // A job's last pixel is done: a staged feed counts it for its tile (the film's sample counts are the host's
  // per-tile job counts, vpt_gpu_feed_snapshot / _collect).  Once per job (64 samples); a uniform branch.
  __device__ __forceinline__ void job_end(const DevScene& S, const LaneCold& lc) {
    uint32_t* const tile_done = Feed ? args()->tile_done : nullptr;
    if (Feed && tile_done)
      atomicAdd(tile_done + (uint32_t)(lc.y0 / S.th) * S.ntx + (uint32_t)(lc.x0 / S.tw), 1u);
  }
  // The film's X, Y, Z: three fp32 adds per sample (the sample-count channel is added per launch by
  // vpt_count_kernel, or per job in a staged feed).  Float atomics execute at the memory side, one request per
  // 64-B line a wave-instruction touches: three instructions whose 64 lanes add to 64 different pixels are 192
  // requests, ~17x the cost of the same bytes contiguous (MI355X_MICROARCH.md § Global float atomics); with
  // them C3 took 348 ms against 328 without any film writes, C4 97 against 77 (r05ab7).  So the kernels with
  // the lane state in LDS regroup a finish pass's samples: film_add only ranks the lane in g_film_rank, and
  // film_commit, run by the converged wavefront, has lane 3k + c add component c of the k-th sample -- one
  // wave-instruction carries 21 samples, each sample's three adds one request.  The latency kernel (state in
  // VGPRs, few samples at a time) adds from the lane itself.
  //
  // The ordered film (args()->samples, vpt_gpu_set_film_order): each lane stores its sample's L into the
  // launch's sample buffer itself -- job j's pixel q at (j * tile_area + q) * 3, j = the job's index in the launch
  // (the cold state's item_lo, set at its fetch) -- and the film is written only by vpt_film_order_kernel, in
  // wave order.  Plain stores complete in the L2 and need no regroup: stored from the lane they measured faster
  // than regrouped through the wavefront as the atomics are (C3 336.1 vs 337.9 ms, C4 81.2 vs 84.2; r06f,
  // profiles/r06f_ordered_direct_and_ray_gate_ab.txt).  (The early return and film_commit's store branch stay as
  // measured: equivalent rewrites of these lines moved the temperature kernel from 0 to 12 bytes of spills.)
  __device__ __forceinline__ bool film_regroup(const DevScene& S) const {
    if (args()->samples) return false;
    return !RegCold && (args()->samples != nullptr || (uint64_t)S.W * (uint64_t)S.H < (1ULL << 26));  // (index << 6 | lane fits 32 bits)
  }
  __device__ __forceinline__ void film_add(const DevScene& S, const Lane& ln, int32_t px, int32_t py, int32_t rw) {
    const LaneCold& lc = cold();
    if constexpr (Feed) {  // the ordered frame's copy of the sample (the film's atomics below stay: the progressive film)
      const uint64_t a = ((uint64_t)lc.item_hi << 32) | lc.item_lo;
      if (args()->frame && a) {
        float* s = reinterpret_cast<float*>(a) + (uint32_t)((py - lc.y0) * rw + (px - lc.x0)) * 3;
        s[0] = lc.L[0];
        s[1] = lc.L[1];
        s[2] = lc.L[2];
      }
    }
    float* const samples = args()->samples;
    const uint32_t pixel = samples ? (uint32_t)((py - lc.y0) * rw + (px - lc.x0)) : (uint32_t)py * (uint32_t)S.W + (uint32_t)px;
    if (film_regroup(S)) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(true);  // this pass's finishing lanes
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      g_film_rank[(threadIdx.x & ~63u) + rank] = (pixel << 6) | (threadIdx.x & 63u);
    } else if (samples) {  // (the ordered film: from the lane itself)
      float* s = samples + ((uint64_t)lc.item_lo * S.tile_area + pixel) * 3;
      s[0] = lc.L[0];
      s[1] = lc.L[1];
      s[2] = lc.L[2];
    } else {
      float* f = args()->film + (uint64_t)pixel * 4;
      const float r = S.imaging_ratio;
      atomicAdd(f + 0, r * lc.L[0]);
      atomicAdd(f + 1, r * lc.L[1]);
      atomicAdd(f + 2, r * lc.L[2]);
    }
#ifdef VPT_JOB_LOG
    if (false) {
#else
    if (float* const records = args()->records) {
#endif
      const int32_t xl = px - lc.x0, yl = py - lc.y0;
      float* rec = args()->records + (ln.jid_local * (uint64_t)args()->tile_area + (uint64_t)(yl * rw + xl)) * 3;
      rec[0] = lc.L[0];
      rec[1] = lc.L[1];
      rec[2] = lc.L[2];
    }
  }
  // fin: this lane ran film_add in the pass just ended.  Called by every lane still in the loop; the lanes that
  // have left it (their jobs done) are not there to add, so the 3 n adds go to the active lanes by rank, as many
  // per wave-instruction as there are active lanes (adds 3k, 3k + 1, 3k + 2: sample k's X, Y, Z).
  __device__ __forceinline__ void film_commit(const DevScene& S, bool fin) {
    if (!film_regroup(S)) return;
    const uint64_t m = __builtin_amdgcn_ballot_w64(fin);
    if (m == 0) return;
    const uint64_t a = __builtin_amdgcn_ballot_w64(true);
    const uint32_t adds = 3u * (uint32_t)__popcll(m), na = (uint32_t)__popcll(a);
    const uint32_t ai = __builtin_amdgcn_mbcnt_hi((uint32_t)(a >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)a, 0u));
    float* const film = args()->film;
    float* const samples = args()->samples;
    const float r = S.imaging_ratio;
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // (else tid & ~63 is hoisted out of the state-machine loop into a VGPR)
    const uint32_t w0 = tid & ~63u;
    for (uint32_t i0 = 0; i0 < adds; i0 += na) {  // (uniform)
      const uint32_t i = i0 + ai;
      if (i < adds) {
        const uint32_t k = i / 3u, c = i - 3u * k;
        const uint32_t e = g_film_rank[w0 + k];
        const LaneCold& src = g_lane_cold[w0 + (e & 63u)];
        if (samples)
          samples[((uint64_t)src.item_lo * S.tile_area + (e >> 6)) * 3 + c] = src.L[c];
        else
          atomicAdd(film + (uint64_t)(e >> 6) * 4 + c, r * src.L[c]);
      }
    }
  }
};


// ---- live-path compaction (north_star: "wavefront ballot/prefix-sum to compact live rays") ----
// The latency kernel's partly filled launches (C2: 2 blocks per CU, 2 jobs per lane) are issue-bound on
// divergent wave instructions: the HDDA step takes 85 % of the wave time and runs at 32.5 of 64 lanes, and per
// walk-loop iteration a wavefront holds 32.7 walking, 14.9 parked (a collision waiting for its batched
// evaluation) and 12.5 finished paths (r05f census, profiles/archive/r05f_c2_census.txt).  Every `compact_every` outer
// iterations the block's four wavefronts meet (two barriers), count their walking / other live paths with
// ballots, and -- when packing would leave fewer wavefronts holding walkers, or live paths -- move every path
// (its hot Lane registers and its cold state, which this kernel keeps in VGPRs: 54 words, 58 with a temperature grid) through LDS so
// that walkers fill the block's first wavefronts, the other live paths the next, finished ones the last.  A
// wavefront without a live path skips its iterations until the next meeting; the block ends when none is left.
// A path's operations and draws never depend on the thread that runs it (its RNG state and every value it reads
// travel with it; the gates only choose when a block runs), so samples are bit-identical; only the order of the
// film's fp32 atomics changes.  The HDDA step counter stays with the thread (it is summed per launch).
constexpr int kXWords = 60;  // 54 state words (58 with a temperature grid), padded to uint4
__device__ __forceinline__ uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
template <bool HasTemp>
__device__ __forceinline__ void xchg_pack(const Lane& ln, const LaneCold& lc, uint32_t x[kXWords]) {
  int n = 0;
  x[n++] = (uint32_t)ln.state; x[n++] = (uint32_t)ln.sm; x[n++] = (uint32_t)ln.shadow;
  x[n++] = (uint32_t)ln.rng; x[n++] = (uint32_t)(ln.rng >> 32);
  for (int i = 0; i < 3; ++i) {
    x[n++] = f2u(ln.e[i]); x[n++] = f2u(ln.d[i]); x[n++] = f2u(ln.nxt[i]);
    x[n++] = (uint32_t)ln.vox[i]; x[n++] = f2u(ln.finc[i]); x[n++] = (uint32_t)ln.vinc[i];
  }
  x[n++] = f2u(ln.scale); x[n++] = f2u(ln.rscale); x[n++] = f2u(ln.maj); x[n++] = (uint32_t)ln.dim;
  x[n++] = f2u(ln.Tn); x[n++] = f2u(ln.T1); x[n++] = ln.pw; x[n++] = f2u(ln.s_t0); x[n++] = f2u(ln.s_t1);
  x[n++] = f2u(ln.s_dmaj);
  x[n++] = (uint32_t)lc.x0; x[n++] = (uint32_t)lc.y0; x[n++] = (uint32_t)lc.pix; x[n++] = lc.depth;
  for (int i = 0; i < 3; ++i) { x[n++] = f2u(lc.L[i]); x[n++] = f2u(lc.ro[i]); x[n++] = f2u(lc.rd[i]); }
  x[n++] = (uint32_t)lc.dens_cell.i; x[n++] = (uint32_t)lc.dens_cell.j; x[n++] = (uint32_t)lc.dens_cell.k;
  x[n++] = (uint32_t)lc.dens_cell.code; x[n++] = f2u(lc.Tr); x[n++] = f2u(lc.y_draw); x[n++] = lc.item_lo;
  x[n++] = lc.item_hi;
  if (HasTemp) {
    x[n++] = (uint32_t)ln.temp_cell.i; x[n++] = (uint32_t)ln.temp_cell.j; x[n++] = (uint32_t)ln.temp_cell.k;
  }
  if (HasTemp) x[n++] = (uint32_t)ln.temp_cell.code;
#ifdef VPT_JOB_LOG
  x[n++] = lc.t_start;  // (the diagnostic build's per-job fields travel too)
  x[n++] = lc.job;
#endif
  while (n < kXWords) x[n++] = 0;
}
static_assert(54 + 4 + 2 <= kXWords, "the exchange holds every state word (and the job log's two)");
template <bool HasTemp>
__device__ __forceinline__ void xchg_unpack(Lane& ln, LaneCold& lc, const uint32_t x[kXWords]) {
  int n = 0;
  ln.state = (int32_t)x[n++]; ln.sm = (int32_t)x[n++]; ln.shadow = (int32_t)x[n++];
  ln.rng = (uint64_t)x[n] | ((uint64_t)x[n + 1] << 32);
  n += 2;
  for (int i = 0; i < 3; ++i) {
    ln.e[i] = u2f(x[n++]); ln.d[i] = u2f(x[n++]); ln.nxt[i] = u2f(x[n++]);
    ln.vox[i] = (int32_t)x[n++]; ln.finc[i] = u2f(x[n++]); ln.vinc[i] = (int32_t)x[n++];
  }
  ln.scale = u2f(x[n++]); ln.rscale = u2f(x[n++]); ln.maj = u2f(x[n++]); ln.dim = (int32_t)x[n++];
  ln.Tn = u2f(x[n++]); ln.T1 = u2f(x[n++]); ln.pw = x[n++]; ln.s_t0 = u2f(x[n++]); ln.s_t1 = u2f(x[n++]);
  ln.s_dmaj = u2f(x[n++]);
  lc.x0 = (int32_t)x[n++]; lc.y0 = (int32_t)x[n++]; lc.pix = (int32_t)x[n++]; lc.depth = x[n++];
  for (int i = 0; i < 3; ++i) { lc.L[i] = u2f(x[n++]); lc.ro[i] = u2f(x[n++]); lc.rd[i] = u2f(x[n++]); }
  lc.dens_cell.i = (int32_t)x[n++]; lc.dens_cell.j = (int32_t)x[n++]; lc.dens_cell.k = (int32_t)x[n++];
  lc.dens_cell.code = (int32_t)x[n++]; lc.Tr = u2f(x[n++]); lc.y_draw = u2f(x[n++]); lc.item_lo = x[n++];
  lc.item_hi = x[n++];
  if (HasTemp) {
    ln.temp_cell.i = (int32_t)x[n++]; ln.temp_cell.j = (int32_t)x[n++]; ln.temp_cell.k = (int32_t)x[n++];
  }
  if (HasTemp) ln.temp_cell.code = (int32_t)x[n++];
#ifdef VPT_JOB_LOG
  lc.t_start = x[n++];
  lc.job = x[n++];
#endif
  (void)n;
}
// Dynamic LDS of the compacting kernel: [kXWords / 4][kBlockThreads] uint4 (61 440 B).
constexpr size_t kXchgBytes = (size_t)kXWords * kBlockThreads * sizeof(uint32_t);

template <bool HasTemp, bool Runs>
__device__ __forceinline__ void compact_loop(ScenePtr sp, Lane& ln, LaneCold& lc, KernelEnvT<true>& env) {
  extern __shared__ uint4 g_xchg[];
  __shared__ int32_t cnt[8];  // per wavefront: walking paths, other live paths
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint64_t below = l ? (~0ULL >> (64 - l)) : 0ULL;
  const uint32_t every = env.args()->compact_every;
  for (;;) {
    for (uint32_t it = 0; it < every; ++it) {
      if (__builtin_amdgcn_ballot_w64(ln.state != ST_DONE) == 0) break;  // (wave-uniform)
      if (ln.state != ST_DONE) lane_iteration<HasTemp, false, Runs>(sp, ln, env);
    }
    const bool walking = ln.state == ST_SAMPLE && ln.sm != SM_EVAL, live = ln.state != ST_DONE;
    const uint64_t mw = __builtin_amdgcn_ballot_w64(walking), mo = __builtin_amdgcn_ballot_w64(live && !walking);
    if (l == 0) {
      cnt[w] = __popcll(mw);
      cnt[4 + w] = __popcll(mo);
    }
    __syncthreads();
    int32_t nw = 0, no = 0, pw = 0, po = 0, pd = 0, wave_w = 0, wave_l = 0;
#pragma unroll
    for (uint32_t v = 0; v < 4; ++v) {
      const int32_t a = cnt[v], b = cnt[4 + v];
      nw += a;
      no += b;
      wave_w += a > 0;
      wave_l += a + b > 0;
      if (v < w) {
        pw += a;
        po += b;
        pd += 64 - a - b;
      }
    }
    if (nw + no == 0) break;  // the block's paths are all done (uniform)
    // exchange only when packing leaves fewer wavefronts with walkers, or with live paths (uniform)
    if ((nw + 63) / 64 < wave_w || (nw + no + 63) / 64 < wave_l) {
      const int32_t dest = walking ? pw + __popcll(mw & below)
                                   : live ? nw + po + __popcll(mo & below) : nw + no + pd + __popcll(~(mw | mo) & below);
      uint32_t x[kXWords];
      xchg_pack<HasTemp>(ln, lc, x);
#pragma unroll
      for (int q = 0; q < kXWords / 4; ++q)
        g_xchg[q * kBlockThreads + dest] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < kXWords / 4; ++q) {
        const uint4 v = g_xchg[q * kBlockThreads + threadIdx.x];
        x[4 * q] = v.x;
        x[4 * q + 1] = v.y;
        x[4 * q + 2] = v.z;
        x[4 * q + 3] = v.w;
      }
      xchg_unpack<HasTemp>(ln, lc, x);
      env.tally(CNT_EXCHANGED, 1);
    }
    __syncthreads();  // cnt and g_xchg are rewritten at the next meeting
  }
}

// counters[] order = vpt_counters field order
template <bool HasTemp, bool Debug, bool Runs, bool Lat = false, bool Compact = false, bool Feed = false>
__global__ __launch_bounds__(kBlockThreads, Compact ? 2 : (Lat ? VPT_WAVES_LAT : (Debug ? VPT_WAVES_SLOW : (HasTemp ? VPT_WAVES_TEMP : VPT_WAVES_FAST)))) void vpt_integrate_kernel(KernelArgs args, const DevScene* scene,
                                                                       unsigned long long* counters) {
  (void)args;  // read through KernelEnvT::args()
  if (threadIdx.x < kCounterCount) g_wg_counters[threadIdx.x] = 0;
  if (threadIdx.x < 32) g_logf_tab[threadIdx.x >> 1][threadIdx.x & 1] = math::kLogfTab[threadIdx.x >> 1][threadIdx.x & 1];
  if (HasTemp) {
    const float* bb = scene->bb;
    for (int i = threadIdx.x; i < kBbFloats; i += kBlockThreads) g_bb_lds[i] = bb[i];
  }
  __syncthreads();
#if defined(VPT_PROFILE) || defined(VPT_PROFILE_TIME)
  if (threadIdx.x < PT_COUNT) g_wg_prof[threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x % 64 == 0) g_wg_prof[PT_COUNT + threadIdx.x / 64] = clock64();
#endif
  KernelEnvT<Lat, Feed> env;
  env.reg_cold = nullptr;
  Lane ln;
  lane_init(ln);
  LaneCold lc_reg;
  if constexpr (Lat) env.reg_cold = &lc_reg;
  cold_init(env.cold());
  const ScenePtr sp = (ScenePtr)scene;
  if constexpr (Compact) {
    static_assert(Lat && !Debug, "compaction runs in the latency kernel only");
    compact_loop<HasTemp, Runs>(sp, ln, lc_reg, env);
  } else
  while (ln.state != ST_DONE) {
    lane_iteration<HasTemp, Debug, Runs>(sp, ln, env);
    // Feed mode: a wavefront whose every live lane waits for the host to publish its item sleeps between
    // polls (~27 us), so idle wavefronts do not flood the host link with reads.
    if (Feed &&
        __builtin_amdgcn_ballot_w64(ln.state == ST_FETCH && (env.cold().pix == kFeedPending ||
                                                              env.cold().pix == kFeedWait)) ==
            __builtin_amdgcn_read_exec())
      for (int i = 0; i < 8; ++i) __builtin_amdgcn_s_sleep(127);
  }
  atomicAdd(g_wg_counters + CNT_DDA_STEPS, (unsigned long long)ln.n_dda);
  __syncthreads();
  if (threadIdx.x < kCounterCount && g_wg_counters[threadIdx.x])
    atomicAdd(counters + threadIdx.x, g_wg_counters[threadIdx.x]);
#if defined(VPT_PROFILE) || defined(VPT_PROFILE_TIME)
  if (threadIdx.x < PT_COUNT) atomicAdd(env.args()->prof_buf + 2 * PB_COUNT + threadIdx.x, g_wg_prof[threadIdx.x]);
#endif
}

// The film's sample-count channel for the job range [jid_begin, jid_begin + jid_count): a pixel of
// tile t gains one sample per job t + k*T in the range (only the single_pixel pixel when that mode is
// on, worker.cpp:113-116).  Counts are integers, so adding them at once equals the reference's
// per-sample += 1.0f (exact below 2^24).
__global__ void vpt_count_kernel(const DevScene* scene, float* film, uint64_t jid_begin, uint64_t jid_count) {
  const DevScene& S = *scene;
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (uint64_t)S.W * (uint64_t)S.H) return;
  const int32_t px = (int32_t)(p % (uint64_t)S.W), py = (int32_t)(p / (uint64_t)S.W);
  if (S.single_pixel_enabled && (px != S.sp_x || py != S.sp_y)) return;
  const uint64_t t = (uint64_t)(py / S.th) * S.ntx + (uint64_t)(px / S.tw), T = S.T, end = jid_begin + jid_count;
  // k from ceil((jid_begin - t) / T) (or 0) to the last k with t + k*T < end
  const uint64_t k0 = jid_begin > t ? (jid_begin - t + T - 1) / T : 0;
  if (t >= end || t + k0 * T >= end) return;
  const uint64_t n = (end - 1 - t) / T - k0 + 1;
  atomicAdd(film + p * 4 + 3, (float)n);
}

// The film's sample-count channel of a feed (vpt_gpu_feed_close): a pixel of tile t gains the number of
// its jobs the host pushed, counts[t] (the same integer sums as vpt_count_kernel's).
__global__ void vpt_tile_count_kernel(const DevScene* scene, float* film, const uint32_t* counts) {
  const DevScene& S = *scene;
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (uint64_t)S.W * (uint64_t)S.H) return;
  const int32_t px = (int32_t)(p % (uint64_t)S.W), py = (int32_t)(p / (uint64_t)S.W);
  if (S.single_pixel_enabled && (px != S.sp_x || py != S.sp_y)) return;
  const uint32_t n = counts[(uint64_t)(py / S.th) * S.ntx + (uint64_t)(px / S.tw)];
  if (n) atomicAdd(film + p * 4 + 3, (float)n);
}

// The ordered film (vpt_gpu_set_film_order): adds the samples of the launch's jobs [jid_begin, jid_begin +
// jid_count) into the film pixel by pixel in wave order -- the order the reference's film receives them: a
// tile's waves are handed out one at a time (TileProvider::next waits for the tile's previous wave,
// tile_provider.cpp:40-60) and each job adds its pixels' samples as it traces them (worker.cpp:203-204:
// w += 1, xyz += imaging_ratio * L).  So the film equals the reference's bit for bit, whatever order the
// launch ran its jobs in.  One thread per (tile, local pixel), so a wavefront reads one job's samples as one
// contiguous run (12 B per pixel) per wave; the film's float4 is read and written once.
__global__ void vpt_film_order_kernel(const DevScene* scene, float* film, const float* samples, uint64_t jid_begin,
                                      uint64_t jid_count) {
  const DevScene& S = *scene;
  const uint32_t area = S.tile_area;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S.T * (uint64_t)area) return;
  const uint64_t t = i / area;
  const uint32_t q = (uint32_t)(i - t * area);
  const int32_t x0 = (int32_t)(t % S.ntx) * S.tw, y0 = (int32_t)(t / S.ntx) * S.th;
  const int32_t rw = min(S.W - x0, S.tw), rh = min(S.H - y0, S.th);
  if ((int32_t)q >= rw * rh) return;
  const int32_t yl = (int32_t)q / rw, px = x0 + ((int32_t)q - yl * rw), py = y0 + yl;
  if (S.single_pixel_enabled && (px != S.sp_x || py != S.sp_y)) return;  // (no sample: worker.cpp:113-116)
  const uint64_t T = S.T, end = jid_begin + jid_count;
  const uint64_t k0 = jid_begin > t ? (jid_begin - t + T - 1) / T : 0;
  if (t + k0 * T >= end) return;
  float4* const f = reinterpret_cast<float4*>(film) + ((uint64_t)py * (uint64_t)S.W + (uint64_t)px);
  float4 a = *f;
  const float r = S.imaging_ratio;
  const float* s = samples + ((t + k0 * T - jid_begin) * area + q) * 3;
  const uint64_t step = T * area * 3;
  const uint64_t n = (end - 1 - t) / T - k0 + 1;
#pragma unroll 8
  for (uint64_t k = 0; k < n; ++k, s += step) {
    a.w = a.w + 1.0f;
    a.x = a.x + r * s[0];
    a.y = a.y + r * s[1];
    a.z = a.z + r * s[2];
  }
  *f = a;
}

// The drop-in's ordered frame (vpt_gpu_frame_finish): the samples its feed launches stored for the jobs [jid_lo,
// jid_end) of the frame's tiles [tile_lo, tile_lo + tiles) (slots as KernelArgs::frame), added pixel by pixel in
// wave order onto film (the film before the frame, or zeros): w += 1, xyz += imaging_ratio * L per sample
// (worker.cpp:203-204), as vpt_film_order_kernel.  Every job of those tiles in the range was rendered (one taker
// hands out a contiguous range of job ids, vpt_run.hpp).
__global__ void vpt_frame_order_kernel(const DevScene* scene, float* film, const float* frame, uint64_t w0, uint32_t tile_lo,
                                       uint32_t tiles, uint64_t jid_lo, uint64_t jid_end) {
  const DevScene& S = *scene;
  const uint32_t area = S.tile_area;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)tiles * area) return;
  const uint32_t tb = (uint32_t)(i / area);
  const uint64_t t = tile_lo + tb;
  const uint32_t q = (uint32_t)(i - (uint64_t)tb * area);
  const int32_t x0 = (int32_t)(t % S.ntx) * S.tw, y0 = (int32_t)(t / S.ntx) * S.th;
  const int32_t rw = min(S.W - x0, S.tw), rh = min(S.H - y0, S.th);
  if ((int32_t)q >= rw * rh) return;
  const int32_t yl = (int32_t)q / rw, px = x0 + ((int32_t)q - yl * rw), py = y0 + yl;
  if (S.single_pixel_enabled && (px != S.sp_x || py != S.sp_y)) return;  // (no sample: worker.cpp:113-116)
  const uint64_t T = S.T;
  const uint64_t j0 = jid_lo + (t + T - jid_lo % T) % T;  // the tile's first job >= jid_lo
  if (j0 >= jid_end) return;
  float4* const f = reinterpret_cast<float4*>(film) + ((uint64_t)py * (uint64_t)S.W + (uint64_t)px);
  float4 a = *f;
  const float r = S.imaging_ratio;
  const float* s = frame + (((j0 / T - w0) * tiles + tb) * area + q) * 3;
  const uint64_t step = (uint64_t)tiles * area * 3;
  const uint64_t n = (jid_end - 1 - j0) / T + 1;
#pragma unroll 8
  for (uint64_t k = 0; k < n; ++k, s += step) {
    a.w = a.w + 1.0f;
    a.x = a.x + r * s[0];
    a.y = a.y + r * s[1];
    a.z = a.z + r * s[2];
  }
  *f = a;
}

// The drop-in's seed recovery (include/vpt_run.hpp rng_seed): the reference's RandomNumberGenerator keeps its u32
// seed private (random.hpp:86-115), so the seeds s whose job-0 stream starts with the outputs (a, b) are found by
// trying all 2^32: hash(s, 0) (hash.hpp:20-67; with jid 0 its k term is 0) | 3 is pcg32_fast's state, whose
// output (xsh_rs: (st ^ st >> 22) >> (22 + st >> 61)) is taken before each multiply (pcg_random.hpp).  Each
// thread tries `per_thread` consecutive seeds; a hit (normally one in 2^32) is appended with an atomic.
__global__ void vpt_seed_search_kernel(uint32_t a, uint32_t b, uint32_t per_thread, uint32_t* found, uint32_t* count,
                                       uint32_t cap) {
  constexpr uint64_t m = 0xc6a4a7935bd1e995ULL, mult = 6364136223846793005ULL;
  const uint64_t first = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * per_thread;
  for (uint32_t i = 0; i < per_thread; ++i) {
    const uint64_t s = first + i;
    if (s >> 32) break;
    uint64_t h = s ^ (8ULL * m);
    h *= m;
    h ^= h >> 47;
    h *= m;
    h ^= h >> 47;
    const uint64_t st = h | 3ULL;
    if ((uint32_t)((st ^ (st >> 22)) >> (22 + (uint32_t)(st >> 61))) != a) continue;
    const uint64_t s2 = st * mult;
    if ((uint32_t)((s2 ^ (s2 >> 22)) >> (22 + (uint32_t)(s2 >> 61))) != b) continue;
    const uint32_t k = atomicAdd(count, 1u);
    if (k < cap) found[k] = (uint32_t)s;
  }
}

// Volume::log_majorant_trace (src/volume.cpp:176-192) of one world ray, on one lane: every
// RayMajorantIterator segment as X0,Y0,Z0,X1,Y1,Z1 (density index space), T0,T1 (world), d_maj.
__global__ void vpt_majorant_trace_kernel(const DevScene* scene, float ox, float oy, float oz, float dx, float dy,
                                          float dz, float* rows, int max_rows, int* n_rows) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ScenePtr sp = (ScenePtr)scene;
  const DevScene S = *sp;
  const DevGrid& G = S.density;
  const float o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz};
  Lane ln;
  lane_init(ln);
  int n = 0;
  if (begin_ray(G, ln, o, ray_dir_setup(G, d))) {
    while (ln.s_t1 < ln.T1) {  // RayMajorantIterator::next: segments until the HDDA leaves [t0, t1]
      begin_segment(ln);
      while (!hdda_step(G, ln)) {
      }
      if (n < max_rows) {
        const float w0 = ln.s_t0 * ln.scale, w1 = ln.s_t1 * ln.scale;  // t * idx_to_world_scale()
        float p0[3], p1[3], q0[3], q1[3];
        for (int i = 0; i < 3; ++i) {  // Ray::eval: origin + direction * t
          p0[i] = o[i] + d[i] * w0;
          p1[i] = o[i] + d[i] * w1;
        }
        map_inv(G, p0[0], p0[1], p0[2], q0[0], q0[1], q0[2]);  // world_to_density_index
        map_inv(G, p1[0], p1[1], p1[2], q1[0], q1[1], q1[2]);
        float* row = rows + 9 * n;
        for (int i = 0; i < 3; ++i) {
          row[i] = q0[i];
          row[3 + i] = q1[i];
        }
        row[6] = w0;
        row[7] = w1;
        row[8] = ln.s_dmaj;
      }
      ++n;
    }
  }
  *n_rows = n;
}

// Cost estimate of every tile for the job order (vpt_gpu_set_job_order): the primary rays through
// the tile's centre and its four quadrant centres, each costed as HDDA steps + 4 x the majorant
// optical depth (expected free-flight draws).  Only the scheduling order depends on it.
__global__ void vpt_tile_cost_kernel(const DevScene* scene, float* cost) {
  const DevScene& S = *scene;
  const uint64_t tile = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tile >= S.T) return;
  const DevGrid& G = S.density;
  const int32_t x0 = (int32_t)(tile % S.ntx) * S.tw, y0 = (int32_t)(tile / S.ntx) * S.th;
  const float rw = (float)min(S.W - x0, S.tw), rh = (float)min(S.H - y0, S.th);
  const float fx[5] = {0.5f, 0.25f, 0.75f, 0.25f, 0.75f}, fy[5] = {0.5f, 0.25f, 0.25f, 0.75f, 0.75f};
  float c = 0.0f;
  for (int r = 0; r < 5; ++r) {
    const float rx = (float)x0 + fx[r] * rw, ry = (float)y0 + fy[r] * rh;
    float dv[3];
    for (int i = 0; i < 3; ++i) dv[i] = S.cam_t[i] + (S.cam_L[i * 3] * rx + S.cam_L[i * 3 + 1] * ry);
    const float n = sqrtf(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
    if (!(n > 0.0f)) continue;
    for (int i = 0; i < 3; ++i) dv[i] /= n;
    Lane ln;
    lane_init(ln);
    if (!begin_ray(G, ln, S.cam_pos, ray_dir_setup(G, dv))) continue;
    int steps = 0;
    float tau = 0.0f;
    while (ln.s_t1 < ln.T1 && steps < (1 << 16)) {
      begin_segment(ln);
      bool done;
      do {
        ++steps;
        done = hdda_step(G, ln);
      } while (!done && steps < (1 << 16));
      tau += S.sigma_t * ln.s_dmaj * (ln.s_t1 - ln.s_t0) * ln.scale;
    }
    c += (float)steps + 4.0f * tau;
  }
  cost[tile] = c;
}

}  // namespace vpt
