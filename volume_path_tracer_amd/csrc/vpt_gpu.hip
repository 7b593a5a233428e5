// vpt_gpu.hip — the MI355X (gfx950) integrator kernel and the C ABI around it.
//
// Kernel shape: a persistent grid sized to the device's resident capacity.  Every lane runs the
// state machine of vpt_integrator.h; when its (tile, wave) job ends it takes the next job id from
// a device counter (one returning atomic per job; the compiler merges a wavefront's simultaneous
// fetches into one atomic), so lanes are refilled until the job range is drained and every wave
// reaches ST_DONE.  Film accumulation uses no-return fp32 atomics into the [H][W][4] XYZW film.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <atomic>
#include <mutex>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "vpt_internal.h"

namespace vpt {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define VPT_HIP(call)                                                                                 \
  do {                                                                                                \
    hipError_t e_ = (call);                                                                           \
    if (e_ != hipSuccess)                                                                             \
      return ::vpt::set_error(VPT_E_HIP, std::string(#call " failed: ") + hipGetErrorString(e_));            \
  } while (0)

constexpr int kCounterCount = CNT_COUNT;
constexpr int kBlockThreads = 256;
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
// Feed mode (vpt_gpu_feed_*): the published word's closed bit, an empty ring slot, a lane's "item
// reserved, not yet published" and "waiting, nothing reserved" marks (LaneCold::pix), and how long a lane
// waits before it gives up (s_memrealtime ticks at 100 MHz: 30 s).
constexpr uint64_t kFeedClosed = 1ULL << 63;
constexpr uint64_t kFeedEmpty = ~0ULL;
constexpr int32_t kFeedPending = -2;
constexpr int32_t kFeedWait = -3;
constexpr uint32_t kFeedDeadline = 3000000000u;
// A waiting wavefront stores the job count it sees again every kWaitingRefresh ticks (~5 ms) while it waits: a
// posted write of an older count may land after a newer one, and the refresh overwrites it.
constexpr uint32_t kWaitingRefresh = 1u << 19;
// Every kStartedHint-th reserved item is reported to the host (the feed's backlog, vpt_gpu_feed_backlog):
// one posted write per 1 024 jobs.
constexpr uint64_t kStartedHint = 1024;
// The hints go to kHintSlots words, item k's to slot (k / kStartedHint) % kHintSlots, and the host takes their
// maximum.  One shared word is not enough: the lanes' posted writes land in any order, so after a burst of
// reservations (a launch's first lane's worth reserves within microseconds) the word could keep an early
// hint for good, and a host that saw the backlog as full would never push again -- r05q: the launch's
// 393 216 items all reserved, the word left at 220 160, the pusher waiting for a backlog of 173 056 to drain
// while every lane waited for it.  Writes to one slot are kHintSlots x kStartedHint items apart.  (16 slots past the word's line measured slower: r05t.)
constexpr uint64_t kHintSlots = 4;
constexpr uint64_t kFeedHeaderWords = 8;  // word, error, waiting, padding, the hint slots [4, 8); then the ring
static_assert(4 + kHintSlots <= kFeedHeaderWords, "the hints fit the header");
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
  // profiles/r02g_c1_lanes_sweep.txt), 1 / 2 / 3 lanes: 8 spp (x = 1.1) 23.3 / 29.3 / - ms, 16 spp
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
  // The ordered film (args()->samples, vpt_gpu_set_film_order): the same regroup with plain stores of each
  // sample's L into the launch's sample buffer (job j's pixel q at (j * tile_area + q) * 3: three lanes store one
  // sample's 12 contiguous bytes, one request), the rank word holding (q << 6) | lane and the job index coming
  // from the source lane's cold state (item_lo, set at its fetch); the film itself is written only by
  // vpt_film_order_kernel, in wave order.
  __device__ __forceinline__ bool film_regroup(const DevScene& S) const {
    return !RegCold && (args()->samples != nullptr || (uint64_t)S.W * (uint64_t)S.H < (1ULL << 26));  // (index << 6 | lane fits 32 bits)
  }
  __device__ __forceinline__ void film_add(const DevScene& S, const Lane& ln, int32_t px, int32_t py, int32_t rw) {
    const LaneCold& lc = cold();
    float* const samples = args()->samples;
    const uint32_t pixel = samples ? (uint32_t)((py - lc.y0) * rw + (px - lc.x0)) : (uint32_t)py * (uint32_t)S.W + (uint32_t)px;
    if (film_regroup(S)) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(true);  // this pass's finishing lanes
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      g_film_rank[(threadIdx.x & ~63u) + rank] = (pixel << 6) | (threadIdx.x & 63u);
    } else if (samples) {  // (the latency kernel: from the lane itself)
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
// evaluation) and 12.5 finished paths (r05f census, profiles/r05f_c2_census.txt).  Every `compact_every` outer
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

// ------------------------------------------------------------------------------------------------
struct DeviceGrid {
  void* cells8 = nullptr;
  void* runs8 = nullptr;
  void* walk8 = nullptr;
  double run_fraction = 0.0;
  void* cells128 = nullptr;
  void* root = nullptr;
  void* bricks = nullptr;
  DevGrid dev{};
  size_t bytes = 0;
};

static int upload(const void* src, size_t n, void** dst, size_t& bytes) {
  *dst = nullptr;
  if (n == 0) return VPT_OK;
  VPT_HIP(hipMalloc(dst, n));
  VPT_HIP(hipMemcpy(*dst, src, n, hipMemcpyHostToDevice));
  bytes += n;
  return VPT_OK;
}

static int upload_grid(const HostGrid& h, DeviceGrid& d) {
  d.dev = h.dev;
  int rc;
  // The stencil pool is 9 KiB per leaf (4.5x the voxels): a large sparse volume can exceed the
  // device's memory.  Say so before the first allocation instead of failing inside hipMalloc.
  const size_t need = h.cells8.size() * sizeof(int2) + h.runs8.size() + h.walk8.size() * sizeof(uint32_t) +
                      h.cells128.size() * sizeof(int2) + h.root.size() * sizeof(RootTileDev) +
                      h.bricks.size() * sizeof(float);
  size_t free_b = 0, total_b = 0;
  VPT_HIP(hipMemGetInfo(&free_b, &total_b));
  if (need > free_b)
    return set_error(VPT_E_NOMEM, "grid upload: needs " + std::to_string(need >> 20) + " MiB (" +
                                      std::to_string(h.dev.leaf_count) + " leaves x 9 KiB stencil pool + tables), " +
                                      std::to_string(free_b >> 20) + " MiB free on the device");
  if ((rc = upload(h.cells8.data(), h.cells8.size() * sizeof(int2), &d.cells8, d.bytes))) return rc;
  if ((rc = upload(h.runs8.data(), h.runs8.size(), &d.runs8, d.bytes))) return rc;
  if ((rc = upload(h.walk8.data(), h.walk8.size() * sizeof(uint32_t), &d.walk8, d.bytes))) return rc;
  d.run_fraction = h.run_fraction;
  if ((rc = upload(h.cells128.data(), h.cells128.size() * sizeof(int2), &d.cells128, d.bytes))) return rc;
  if ((rc = upload(h.root.data(), h.root.size() * sizeof(RootTileDev), &d.root, d.bytes))) return rc;
  if ((rc = upload(h.bricks.data(), h.bricks.size() * sizeof(float), &d.bricks, d.bytes))) return rc;
  d.dev.cells8 = (const int2*)d.cells8;
  d.dev.runs8 = (const uint8_t*)d.runs8;
  d.dev.walk8 = (const uint32_t*)d.walk8;
  d.dev.cells128 = (const int2*)d.cells128;
  d.dev.root = (const RootTileDev*)d.root;
  d.dev.bricks = (const float*)d.bricks;
  return VPT_OK;
}

static void free_grid(DeviceGrid& d) {
  (void)hipFree(d.cells8);
  (void)hipFree(d.runs8);
  (void)hipFree(d.walk8);
  (void)hipFree(d.cells128);
  (void)hipFree(d.root);
  (void)hipFree(d.bricks);
  d = DeviceGrid{};
}

}  // namespace vpt

namespace vpt {
// The shared state of an open feed, as its launch sees it (see KernelEnvT::fetch_feed).
struct FeedLaunch {
  const uint64_t* word;
  uint64_t* ring;
  uint64_t mask;
  unsigned* error;
  uint64_t* started;
  uint64_t* waiting;
  uint32_t* tile_done;  // nullptr unless a staged feed
};
}  // namespace vpt

struct vpt_gpu_feed;

struct vpt_gpu_ctx {
  int device = 0;
  vpt_configuration cfg{};
  vpt::DevScene scene{};
  vpt::DeviceGrid density, temperature;
  float* bb = nullptr;
  float* cie = nullptr;
  float* film = nullptr;
  uint64_t film_count = 0;
  // Per-launch job / event counters: a ring of kLaunchSlots pairs, so launches on different streams
  // of one context never share a counter.  slot_done[i] is recorded on the stream of the launch
  // that last used slot i; the next launch to take slot i waits for it on its own stream first.
  unsigned long long* job_counter = nullptr;  // [kLaunchSlots][2]: jobs, events
  hipEvent_t slot_done[64] = {};
  bool slot_used[64] = {};
  uint32_t next_slot = 0;
  std::mutex slot_mu;
  unsigned long long* counters = nullptr;
  unsigned long long* prof = nullptr;
  vpt::DevScene* scene_dev = nullptr;  // the kernel's copy of scene (read through ScenePtr)
  // Latency-bound launches (fewer work items than the grid has lanes): their own gates (a second
  // device copy of the scene with lat_gate[] in place of the gates) and jobs spread over wavefronts.
  vpt::DevScene* scene_lat_dev = nullptr;
  int lat_gate[4] = {1, 65, 1, 1};   // gate_min, gate_idle, gate_eval, gate_walk
  int lat_wave_lanes = 0;            // 0: spread the items evenly over the grid's wavefronts
  hipStream_t stream = nullptr;
  bool use_runs = false;             // density-only kernel variant with run skipping (see create)
  int pixel_chunk = 0;               // throughput mode: pixels per work item (0 = auto, see render)
  int grid_blocks = 0;               // resident capacity (or the set_tuning override)
  int cus = 1;                       // compute units of the device
  bool grid_user = false;            // grid_blocks set by vpt_gpu_set_tuning: use it as is
  int order_mode = VPT_ORDER_COST_TAIL;
  int order_tail_waves = 0;        // VPT_ORDER_COST_TAIL: tile-major waves (0 = auto)
  uint32_t* order = nullptr;       // tile ranks by descending cost (device), built on first use
  std::vector<float> tile_cost;    // host copy of the estimates
  uint32_t* perm = nullptr;        // explicit job order of launches with perm_n jobs (device)
  uint64_t perm_n = 0;
  std::vector<uint32_t> tile_rank;
  float* staging = nullptr;        // pinned host buffer of film_count floats (vpt_gpu_film_flush_to_host)
  // Feeds whose launches have ended, kept for reuse: while a feed is open its launch holds the device,
  // and a call that waits for the whole device (hipFree, hipHostFree, hipHostMalloc may) would wait for
  // that launch -- i.e. until its lanes give up -- so a feed's memory is allocated once and freed with
  // the context.
  std::vector<vpt_gpu_feed*> feed_pool;
  // Feeds launched and not yet closed: a call that waits for the context's launches (wait_ctx) would wait
  // for such a feed's lanes to give up (30 s) and lose its work, so those calls refuse while it is > 0.
  std::atomic<int> open_feeds{0};
  // Pinned zeros: staged feeds clear their film and tile counts with host-to-device copies, which the copy
  // engines run beside a launch that holds every CU (a fill kernel would wait for it; r05a probe).
  float* zeros = nullptr;
  int lat_mode = -1;              // latency kernel: -1 auto (launches of <= lat_per_cu blocks per CU), 0 off, 1 on
  int lat_ungated = 0;             // its partly filled launches read the latency gates (1) or the context's (0)
  int lat_per_cu = 1;              // resident blocks per CU of the latency kernel
  int compact_every = 0;           // live-path compaction on partly filled latency launches: meeting period (0 off)
  int compact_per_cu = 0;          // resident blocks per CU of the compacting kernel (its LDS exchange)
  // The ordered film (vpt_gpu_set_film_order): the sample buffer of ordered launches (one at a time: each
  // waits for the previous one's vpt_film_order_kernel, samples_done), and the largest buffer a launch may use
  // (0 = auto, 3/4 of the device's free memory when it grows; larger launches are split).
  int film_order = VPT_FILM_ORDERED;
  uint64_t film_order_max = 0;
  float* samples = nullptr;
  uint64_t samples_bytes = 0;
  hipEvent_t samples_done = nullptr;
  bool samples_used = false;
  uint64_t ordered_launches = 0, atomic_launches = 0;  // (vpt_gpu_film_order_info)
  // vpt_gpu_create's phases (ms): grid flatten + majorant fix, grid upload, the rest, the tile-cost pass, device bind
  double setup_ms[5] = {};
};

namespace {

constexpr int kProfWords = 2 * vpt::PB_COUNT + vpt::PT_COUNT;
constexpr uint32_t kLaunchSlots = 64;
// Latency-bound launches: at most this many work items per wavefront of the grid (see render()).
constexpr uint64_t kSpreadLanes = 6;

int ctx_device(vpt_gpu_ctx* ctx);
int wait_ctx(vpt_gpu_ctx* ctx);

// Device copy of the scene constants, which every in-flight launch of this context reads: wait for
// the context's launches (wait_ctx), copy on the context's stream and wait for the copy (the next
// render may use another stream).
int push_scene(vpt_gpu_ctx* ctx) {
  int rc = wait_ctx(ctx);
  if (rc) return rc;
  vpt::DevScene lat = ctx->scene;
  lat.gate_min = ctx->lat_gate[0];
  lat.gate_idle = ctx->lat_gate[1];
  lat.gate_eval = ctx->lat_gate[2];
  lat.gate_walk = ctx->lat_gate[3];
  lat.wave_lanes = ctx->lat_wave_lanes;
  VPT_HIP(hipMemcpyAsync(ctx->scene_dev, &ctx->scene, sizeof(vpt::DevScene), hipMemcpyHostToDevice, ctx->stream));
  VPT_HIP(hipMemcpyAsync(ctx->scene_lat_dev, &lat, sizeof(vpt::DevScene), hipMemcpyHostToDevice, ctx->stream));
  VPT_HIP(hipStreamSynchronize(ctx->stream));
  return VPT_OK;
}

// The counter pair of the next launch on stream s: ordered after the previous launch that used the
// same ring slot (whatever stream it ran on), then zeroed on s.
int take_slot(vpt_gpu_ctx* ctx, hipStream_t s, uint32_t& slot) {
  std::lock_guard<std::mutex> lock(ctx->slot_mu);
  slot = ctx->next_slot;
  ctx->next_slot = (ctx->next_slot + 1) % kLaunchSlots;
  if (ctx->slot_used[slot]) VPT_HIP(hipStreamWaitEvent(s, ctx->slot_done[slot], 0));
  VPT_HIP(hipMemsetAsync(ctx->job_counter + 2 * slot, 0, 2 * sizeof(unsigned long long), s));
  return VPT_OK;
}

int release_slot(vpt_gpu_ctx* ctx, hipStream_t s, uint32_t slot) {
  std::lock_guard<std::mutex> lock(ctx->slot_mu);
  VPT_HIP(hipEventRecord(ctx->slot_done[slot], s));
  ctx->slot_used[slot] = true;
  return VPT_OK;
}

// Waits for every launch of this context, whatever stream it was enqueued on, and for the context's
// own stream -- not for other contexts' work on the device (a context per thread never stalls
// behind another's frames).  Each launch records its ring slot's event after its kernels
// (release_slot), and a launch that reuses a slot is ordered after the slot's previous launch
// (take_slot), so the latest event of every used slot covers all of them.
// The events are snapshotted under the lock and waited for after it is released, so a wait never
// blocks another thread's take_slot.
int wait_ctx(vpt_gpu_ctx* ctx) {
  if (ctx->open_feeds.load() > 0)
    return vpt::set_error(VPT_E_STATE, "a feed of this context is open: close it before calls that wait for the "
                                       "context's launches (ADVICE r04)");
  hipEvent_t ev[kLaunchSlots];
  uint32_t n = 0;
  {
    std::lock_guard<std::mutex> lock(ctx->slot_mu);
    for (uint32_t i = 0; i < kLaunchSlots; ++i)
      if (ctx->slot_used[i]) ev[n++] = ctx->slot_done[i];
  }
  for (uint32_t i = 0; i < n; ++i) VPT_HIP(hipEventSynchronize(ev[i]));
  if (ctx->stream) VPT_HIP(hipStreamSynchronize(ctx->stream));
  return VPT_OK;
}

int ctx_device(vpt_gpu_ctx* ctx) {
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return VPT_OK;
}

void feed_pool_free(vpt_gpu_ctx* ctx);

void destroy(vpt_gpu_ctx* ctx) {
  if (!ctx) return;
  feed_pool_free(ctx);
  (void)hipSetDevice(ctx->device);
  vpt::free_grid(ctx->density);
  vpt::free_grid(ctx->temperature);
  (void)hipFree(ctx->bb);
  (void)hipFree(ctx->cie);
  (void)hipFree(ctx->film);
  (void)hipFree(ctx->job_counter);
  (void)hipFree(ctx->counters);
  (void)hipFree(ctx->prof);
  (void)hipFree(ctx->scene_dev);
  (void)hipFree(ctx->scene_lat_dev);
  (void)hipFree(ctx->order);
  (void)hipFree(ctx->perm);
  (void)hipFree(ctx->samples);
  if (ctx->samples_done) (void)hipEventDestroy(ctx->samples_done);
  for (uint32_t i = 0; i < kLaunchSlots; ++i)
    if (ctx->slot_done[i]) (void)hipEventDestroy(ctx->slot_done[i]);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->staging) (void)hipHostFree(ctx->staging);
  delete ctx;
}

// The descending-cost tile ranks of ctx->tile_cost, uploaded as the job order.
int rank_tiles(vpt_gpu_ctx* ctx) {
  const uint64_t T = ctx->scene.T;
  ctx->tile_rank.resize(T);
  for (uint64_t i = 0; i < T; ++i) ctx->tile_rank[i] = (uint32_t)i;
  std::stable_sort(ctx->tile_rank.begin(), ctx->tile_rank.end(),
                   [&](uint32_t a, uint32_t b) { return ctx->tile_cost[a] > ctx->tile_cost[b]; });
  uint32_t* d = nullptr;
  VPT_HIP(hipMalloc((void**)&d, T * sizeof(uint32_t)));
  const hipError_t e = hipMemcpy(d, ctx->tile_rank.data(), T * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return vpt::set_error(VPT_E_HIP, std::string("tile order upload: ") + hipGetErrorString(e));
  }
  (void)hipFree(ctx->order);
  ctx->order = d;
  return VPT_OK;
}

// Tile costs (vpt_tile_cost_kernel) and the descending-cost tile ranks, once per context.
int ensure_order(vpt_gpu_ctx* ctx) {
  if (ctx->order) return VPT_OK;
  const auto t0 = std::chrono::steady_clock::now();
  struct Lap {  // (the cost pass's time, vpt_gpu_setup_timings)
    vpt_gpu_ctx* c;
    std::chrono::steady_clock::time_point t0;
    ~Lap() { c->setup_ms[3] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
  } lap{ctx, t0};
  if (ctx->open_feeds.load() > 0)  // the cost pass and its copy would wait for the feed's launch
    return vpt::set_error(VPT_E_STATE, "tile costs: a feed of this context is open (compute them before)");
  const uint64_t T = ctx->scene.T;
  float* cost = nullptr;
  VPT_HIP(hipMalloc((void**)&cost, T * sizeof(float)));
  hipLaunchKernelGGL(vpt::vpt_tile_cost_kernel, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, nullptr,
                     ctx->scene_dev, cost);
  ctx->tile_cost.assign(T, 0.0f);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(ctx->tile_cost.data(), cost, T * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(cost);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("tile cost pass: ") + hipGetErrorString(e));
  return rank_tiles(ctx);
}

// The ordered film's sample buffer for a launch of `bytes`: the context's, grown if needed.  nullptr (VPT_OK)
// when it must grow while a feed of the context is open -- freeing or allocating device memory could wait for
// the feed's launch -- and that launch then adds into the film with atomics.
int ensure_samples(vpt_gpu_ctx* ctx, uint64_t bytes, float*& out) {
  out = nullptr;
  if (ctx->samples_bytes >= bytes) {
    out = ctx->samples;
    return VPT_OK;
  }
  if (ctx->open_feeds.load() > 0) return VPT_OK;
  if (ctx->samples_used) VPT_HIP(hipEventSynchronize(ctx->samples_done));  // (ordered launches are serialised)
  if (ctx->samples) {
    (void)hipFree(ctx->samples);
    ctx->samples = nullptr;
    ctx->samples_bytes = 0;
  }
  const hipError_t e = hipMalloc((void**)&ctx->samples, bytes);
  if (e != hipSuccess) {
    ctx->samples = nullptr;
    (void)hipGetLastError();
    return vpt::set_error(VPT_E_NOMEM, "ordered film: " + std::to_string(bytes >> 20) + " MiB sample buffer: " +
                                           hipGetErrorString(e) + " (vpt_gpu_set_film_order's max_bytes splits launches)");
  }
  ctx->samples_bytes = bytes;
  out = ctx->samples;
  return VPT_OK;
}

// The largest sample buffer an ordered launch may use (bytes).
uint64_t ordered_cap(vpt_gpu_ctx* ctx, uint64_t want) {
  if (ctx->film_order_max) return ctx->film_order_max;
  if (want <= ctx->samples_bytes) return ctx->samples_bytes;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return ctx->samples_bytes;
  return (uint64_t)(free_b + ctx->samples_bytes) / 4 * 3;
}

int render(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film, float* records, void* stream_ptr,
           vpt_event* events = nullptr, uint64_t event_cap = 0, uint32_t* slot_out = nullptr,
           const vpt::FeedLaunch* feed = nullptr) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "render: null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if (jid_count == 0) return VPT_OK;
  if (feed && (ctx->scene.pixel_mode || records || events))
    return vpt::set_error(VPT_E_INVALID, "render: feeds run the reference RNG mode's production kernels only");
  // The ordered film: production launches of the reference RNG mode (debug launches and feeds add atomically).
  // A launch whose sample buffer would exceed the cap is rendered as consecutive launches (whole waves where it
  // can); each adds its own waves in order, so the film is the same.
  const uint64_t per_job = (uint64_t)ctx->scene.tile_area * 3 * sizeof(float);
  const bool ordered = ctx->film_order == VPT_FILM_ORDERED && !feed && !records && !events && !ctx->scene.pixel_mode;
  if (ordered) {
    const uint64_t max_jobs = std::min<uint64_t>(ordered_cap(ctx, jid_count * per_job) / per_job, 0xffffffffULL);
    if (max_jobs == 0) return vpt::set_error(VPT_E_NOMEM, "ordered film: no room for one job's samples");
    if (jid_count > max_jobs) {
      const uint64_t T = ctx->scene.T;
      const uint64_t chunk = max_jobs >= T ? max_jobs / T * T : max_jobs;
      for (uint64_t b = 0; b < jid_count; b += chunk)
        if ((rc = render(ctx, jid_begin + b, std::min(chunk, jid_count - b), film, nullptr, stream_ptr))) return rc;
      return VPT_OK;
    }
  }
  const uint64_t total = ctx->scene.T * (uint64_t)ctx->cfg.num_waves;
  (void)total;  // jids beyond num_waves are valid jobs too (TileProvider only stops at requested_waves)
  hipStream_t s = (hipStream_t)stream_ptr;  // NULL = the null stream (HIP convention)
  vpt::KernelArgs env{};
  env.jid_begin = jid_begin;
  env.jid_count = jid_count;
  env.pixel_chunk = 1;
  if (ctx->scene.pixel_mode) {  // work items are chunks of pixel_chunk pixels of one job
    const uint64_t area = ctx->scene.tile_area;
    if (jid_count > UINT64_MAX / area) return vpt::set_error(VPT_E_INVALID, "render: job range too large");
    const uint64_t items = jid_count * area;
    // One work item per pixel makes every pixel a device-wide atomic on the launch's job counter, and a
    // wavefront's fetches then serialise there (C3: 530 M pixels, 546 ms vs 348 in the reference mode,
    // r03zf).  Pixels are taken pixel_chunk at a time: the largest power of two dividing the tile area that
    // still leaves >= 32 chunks per resident lane (C3 / C5: 32 pixels; C2, C1: 1 -- C2 ran 41.6 ms with 1
    // pixel per item, 43.7 with 4, r03zg), or the vpt_gpu_set_pixel_chunk value.  Every pixel keeps its own
    // stream: samples do not depend on it.
    uint64_t K = 1;
    if (ctx->pixel_chunk > 0) {
      K = (uint64_t)ctx->pixel_chunk;
    } else {
      const uint64_t lanes = (uint64_t)ctx->grid_blocks * vpt::kBlockThreads;
      while (area % (2 * K) == 0 && items / (2 * K) >= 32 * lanes) K *= 2;
    }
    env.pixel_chunk = (uint32_t)K;
    env.jid_count = items / K;
  }
  env.film = film ? film : ctx->film;
  env.records = records;
  env.tile_area = ctx->scene.tw * ctx->scene.th;
  env.prof_buf = ctx->prof;
  env.order = nullptr;
  env.perm = nullptr;
  env.order_tail_k0 = 0;
  env.order_tail_n = 0;
  // Partly filled launches (a few work items per resident lane: small frames, few waves, a GPU's share
  // of a frame dealt over several): a launch lasts as long as its slowest jobs, and a job's lane runs
  // faster with fewer waves per SIMD, so the grid is sized to round(1 + 1.8 x) blocks per CU (at most
  // the resident capacity), x = items per resident lane.  Same jobs, same samples.  Measured (r03h,
  // profiles/r03h_grid_sweep.txt; C3 frames of spp waves, 4 / 5 / 6 / 7 blocks per CU, ms): spp 16
  // (x 1.1) 54.5 / 55.0 / 55.4 / 57.5 (3: 51.5); spp 24 (x 1.7) 57.3 / 61.0 / 64.7 / 65.7; spp 32
  // (x 2.3, the 8-GPU share) 70.4 / 66.9 / 67.5 / 71.2; spp 48 (x 3.4) 92.2 / 90.8 / 89.7 / 87.9; from
  // spp 96 on (and C5's shares) the full grid is best.  C2 (262 144 jobs, x 0.57 -> 2 blocks per CU,
  // r02g: 1 / 1.5 / 1.75 / 2 / 2.5 / 3 / 4 / 5 blocks per CU 167.7 / 124.4 / 112.9 / 98.7-99.3 / 104.4 /
  // 104.5-105.3 / 106.7 / 109.9 ms).  (r02's rule, ~2 items per lane, gave 7 blocks from x 1.9 on.)
  uint32_t blocks = (uint32_t)ctx->grid_blocks;
  // Latency-bound launch (at most kSpreadLanes items per wavefront of the grid, e.g. C1's 4 096 jobs):
  // the launch lasts as long as its slowest job, and a job runs fastest on a wavefront with few other
  // paths (the wavefront executes every block any of its lanes needs).  Such a launch keeps the whole
  // grid, the first ~items / wavefronts lanes of each wavefront take the jobs, and it runs with the
  // latency gates (every block runs for one lane).  Measured, C1 (r02): 43.3 ms (256 blocks x 64
  // lanes) -> 20.5 ms (1 792 blocks, one lane per wavefront, gates 1:65:1:1).  Same jobs, same samples.
  const bool latency = env.jid_count <= kSpreadLanes * ((uint64_t)blocks * (vpt::kBlockThreads / 64));
  const uint64_t cus = (uint64_t)ctx->cus;
  if (!ctx->grid_user && !latency) {
    const uint64_t resident_per_cu = std::max<uint64_t>(1, blocks / cus);
    const double x = (double)env.jid_count / ((double)blocks * vpt::kBlockThreads);  // items per resident lane
    const uint64_t per_cu = std::min<uint64_t>(resident_per_cu, (uint64_t)std::max(1.0, std::floor(1.5 + 1.8 * x)));
    blocks = (uint32_t)std::min<uint64_t>(blocks, cus * per_cu);
  }
#ifdef VPT_JOB_LOG
  const bool temp = ctx->scene.has_temperature != 0, dbg = events != nullptr;  // records = the job log
#else
  const bool temp = ctx->scene.has_temperature != 0, dbg = records != nullptr || events != nullptr;
#endif
  // The latency kernel (lane cold state in VGPRs, VPT_WAVES_LAT waves per SIMD) for launches that fill at
  // most its resident grid anyway: latency-bound ones on its whole grid with the latency gates (C1 20.7-21.2
  // -> 19.2-19.7 ms, r04e / r04z), and partly filled ones whose rule above gives <= lat_per_cu blocks per CU
  // with the context's gates (C2 100.0-101.3 -> 95.7-96.6 ms, the 8-GPU C3 share of 32 waves 66.1-66.6 ->
  // 65.1-65.3; with the latency gates they ran slower, 108.3-109.8 / 75.2-76.1 ms: its one-lane blocks add
  // wave instructions to launches that are issue-bound; r04k, profiles/r04k_lat_gated_ab.txt).  lat_mode 1
  // forces it.  Same jobs, same samples.
  const uint64_t lat_blocks = cus * (uint64_t)ctx->lat_per_cu;
  const bool use_lat = !dbg && !feed && ctx->lat_mode != 0 &&
                       (ctx->lat_mode == 1 || (!ctx->grid_user && (latency || blocks <= lat_blocks)));
  if (use_lat) blocks = (uint32_t)std::min<uint64_t>(latency ? lat_blocks : blocks, lat_blocks);
  // Live-path compaction (vpt_gpu_set_compaction): partly filled launches of the latency kernel whose grid fits
  // the compacting kernel's occupancy (its LDS exchange: 2 blocks per CU; C2 runs 2).
  const bool compact = use_lat && !latency && ctx->compact_every > 0 &&
                       (uint64_t)blocks <= cus * (uint64_t)std::max(0, ctx->compact_per_cu);
  const uint64_t T = ctx->scene.T;
  if (!feed && ctx->order_mode != VPT_ORDER_JID && jid_begin % T == 0 && jid_count % T == 0 && jid_count < (1ULL << 32)) {
    // whole waves: take the jobs in cost order (same jobs, same samples)
    if ((rc = ensure_order(ctx))) return rc;
    const uint32_t n = (uint32_t)(jid_count / T);
    uint32_t tail = 0;  // VPT_ORDER_COST_WAVE_MAJOR
    if (ctx->order_mode == VPT_ORDER_COST_TILE_MAJOR) tail = n;
    if (ctx->order_mode == VPT_ORDER_COST_TAIL) {
      // the last ~6 x (resident lanes / T) waves (C3: 61 of 256): measured best of 2x..16x
      const uint64_t lanes = (uint64_t)blocks * vpt::kBlockThreads;
      const uint64_t want = ctx->order_tail_waves > 0 ? (uint64_t)ctx->order_tail_waves : (6 * lanes + T - 1) / T;
      tail = (uint32_t)std::min<uint64_t>(n, want);
    }
    env.order = ctx->order;
    env.order_tail_n = tail;
    env.order_tail_k0 = (n - tail) * (uint32_t)T;
  }
  if (!feed && ctx->perm && ctx->perm_n == jid_count && !ctx->scene.pixel_mode) env.perm = ctx->perm;
  float* samples = nullptr;
  if (ordered && (rc = ensure_samples(ctx, jid_count * per_job, samples))) return rc;
  env.samples = samples;
  if (samples) {
    ++ctx->ordered_launches;
    if (ctx->samples_used) VPT_HIP(hipStreamWaitEvent(s, ctx->samples_done, 0));  // the buffer's previous launch
  } else if (!feed) {
    ++ctx->atomic_launches;
  }
  uint32_t slot = 0;
  if ((rc = take_slot(ctx, s, slot))) return rc;
  env.job_counter = ctx->job_counter + 2 * slot;
  env.events = events;
  env.feed_word = feed ? feed->word : nullptr;
  env.feed_ring = feed ? feed->ring : nullptr;
  env.feed_mask = feed ? feed->mask : 0;
  env.feed_error = feed ? feed->error : nullptr;
  env.feed_started = feed ? feed->started : nullptr;
  env.feed_waiting = feed ? feed->waiting : nullptr;
  env.feed_hint_mask = (uint32_t)(vpt::kHintSlots - 1);
  env.tile_done = feed ? feed->tile_done : nullptr;
  env.compact_every = 0;
  env.event_count = ctx->job_counter + 2 * slot + 1;
  env.event_cap = event_cap;
  if (slot_out) *slot_out = slot;
  // (a compacting launch reads the context's scene, whose wave_lanes is 64: a path moved into another thread's
  // slot must be able to fetch there -- with fewer fetching lanes per wavefront, live paths packed into the
  // first slots would leave the fetching slots to finished ones)
  const vpt::DevScene* scene =
      latency || (use_lat && ctx->lat_ungated && !compact) ? ctx->scene_lat_dev : ctx->scene_dev;
  if (use_lat) {
    env.compact_every = (uint32_t)std::max(1, ctx->compact_every);
    if (compact) {
      auto kernel = temp ? vpt::vpt_integrate_kernel<true, false, false, true, true>
                         : ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true, true>
                                         : vpt::vpt_integrate_kernel<false, false, false, true, true>;
      hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), vpt::kXchgBytes, s, env, scene, ctx->counters);
    } else {
      auto kernel = temp ? vpt::vpt_integrate_kernel<true, false, false, true>
                         : ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true>
                                         : vpt::vpt_integrate_kernel<false, false, false, true>;
      hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), 0, s, env, scene, ctx->counters);
    }
  } else if (feed) {  // (never a debug launch: no records or events)
    auto kernel = temp ? vpt::vpt_integrate_kernel<true, false, false, false, false, true>
                       : ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, false, false, true>
                                       : vpt::vpt_integrate_kernel<false, false, false, false, false, true>;
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), 0, s, env, scene, ctx->counters);
  } else {
    auto kernel = temp ? (dbg ? vpt::vpt_integrate_kernel<true, true, false> : vpt::vpt_integrate_kernel<true, false, false>)
                       : ctx->use_runs
                           ? (dbg ? vpt::vpt_integrate_kernel<false, true, true> : vpt::vpt_integrate_kernel<false, false, true>)
                           : (dbg ? vpt::vpt_integrate_kernel<false, true, false> : vpt::vpt_integrate_kernel<false, false, false>);
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), 0, s, env, scene, ctx->counters);
  }
  VPT_HIP(hipGetLastError());
  const uint64_t npix = (uint64_t)ctx->scene.W * (uint64_t)ctx->scene.H;
  if (samples) {  // the film, pixel by pixel in wave order (sample counts included)
    const uint64_t threads = ctx->scene.T * (uint64_t)ctx->scene.tile_area;
    hipLaunchKernelGGL(vpt::vpt_film_order_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                       ctx->scene_dev, env.film, samples, jid_begin, jid_count);
    VPT_HIP(hipGetLastError());
    VPT_HIP(hipEventRecord(ctx->samples_done, s));
    ctx->samples_used = true;
  } else if (!feed) {  // a feed adds its sample counts when it is closed (vpt_tile_count_kernel)
    hipLaunchKernelGGL(vpt::vpt_count_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, ctx->scene_dev,
                       env.film, jid_begin, jid_count);
    VPT_HIP(hipGetLastError());
  }
  return release_slot(ctx, s, slot);
}

}  // namespace

extern "C" {

const char* vpt_last_error(void) { return vpt::g_last_error.c_str(); }
int vpt_abi_version(void) { return VPT_ABI_VERSION; }

int vpt_gpu_device_count(int* count) {
  if (!count) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_device_count: null argument");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return VPT_OK;
}

int vpt_gpu_find_seeds(int device, uint32_t out0, uint32_t out1, uint32_t* seeds, int max_seeds, int* n_found) {
  if (!n_found || max_seeds < 0 || (max_seeds > 0 && !seeds))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_find_seeds: bad argument");
  *n_found = 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return vpt::set_error(VPT_E_HIP, "vpt_gpu_find_seeds: no HIP device");
  if (device < 0 || device >= ndev) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_find_seeds: bad device index");
  VPT_HIP(hipSetDevice(device));
  constexpr uint32_t kCap = 64, kPerThread = 1024, kThreads = 256;
  hipStream_t s = nullptr;
  VPT_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* d = nullptr;
  uint32_t host[kCap + 1] = {};
  hipError_t e = hipMalloc((void**)&d, (kCap + 1) * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemsetAsync(d, 0, (kCap + 1) * sizeof(uint32_t), s);
  if (e == hipSuccess) {
    const uint64_t blocks = ((1ULL << 32) / kPerThread + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(vpt::vpt_seed_search_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, out0, out1, kPerThread,
                       d + 1, d, kCap);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(host, d, sizeof host, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_find_seeds: ") + hipGetErrorString(e));
  const uint32_t n = std::min(host[0], kCap);
  std::sort(host + 1, host + 1 + n);
  for (uint32_t i = 0; i < n && (int)i < max_seeds; ++i) seeds[i] = host[1 + i];
  *n_found = (int)host[0];
  return VPT_OK;
}

int vpt_gpu_create(const vpt_configuration* cfg, const vpt_grid_desc* density, const vpt_grid_desc* temperature,
                   const float* blackbody_500x3, int device, vpt_gpu_ctx** out) {
  if (!cfg || !density || !out) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_create: null argument");
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0)
    return vpt::set_error(VPT_E_HIP, "vpt_gpu_create: no HIP device (the integrator has no CPU fallback)");
  if (device < 0 || device >= ndev) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_create: bad device index");
  std::unique_ptr<vpt_gpu_ctx, void (*)(vpt_gpu_ctx*)> ctx(new vpt_gpu_ctx(), destroy);
  ctx->device = device;
  ctx->cfg = *cfg;
  using clk = std::chrono::steady_clock;
  auto t = clk::now();
  auto lap = [&](int i) {  // setup phases (vpt_gpu_setup_timings)
    const auto now = clk::now();
    ctx->setup_ms[i] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  };
  int rc = ctx_device(ctx.get());
  if (rc) return rc;
  lap(4);
  if ((rc = vpt::build_scene(*cfg, ctx->scene))) return rc;

  // Volume::Volume: fix the density majorants (volume.cpp:162-170); temperature is only sampled.
  {
    vpt::HostGrid h;
    if ((rc = vpt::build_host_grid(*density, true, 0, h))) return rc;
    vpt::compute_runs(h, 0);
    lap(0);
    if ((rc = vpt::upload_grid(h, ctx->density))) return rc;
    lap(1);
  }
  if (temperature) {
    vpt::HostGrid h;
    if ((rc = vpt::build_host_grid(*temperature, false, 0, h))) return rc;
    lap(0);
    if ((rc = vpt::upload_grid(h, ctx->temperature))) return rc;
    lap(1);
  }
  // The run-skipping kernel variant is for grids with large equal-majorant regions (C2's constant
  // cube: 36 % of the interior cells have run radius >= 2; the 512^3 cloud: 4 %, where the variant
  // would cost more than it skips).  vpt_gpu_set_run_skipping overrides the choice.
  ctx->use_runs = !temperature && ctx->density.run_fraction >= 0.25;
  ctx->scene.density = ctx->density.dev;
  vpt::scene_finalize(ctx->scene);  // uses only the density map (host copy of the values)
  ctx->scene.temperature = ctx->temperature.dev;
  ctx->scene.has_temperature = temperature ? 1 : 0;
  ctx->scene.bb_lds_ok = temperature ? vpt::blackbody_rows_suffice(*temperature, cfg->volume_parameters.temperature_scale,
                                                                    cfg->volume_parameters.temperature_offset, vpt::kBbLdsRows)
                                     : 0;

  std::vector<float> bb(501 * 3, 0.0f);  // row 500 = 0 (reference reads past its table)
  if (blackbody_500x3)
    std::memcpy(bb.data(), blackbody_500x3, 500 * 3 * sizeof(float));
  else
    vpt::blackbody_table(bb.data());
  size_t scratch = 0;
  if ((rc = vpt::upload(bb.data(), bb.size() * sizeof(float), (void**)&ctx->bb, scratch))) return rc;
  if ((rc = vpt::upload(vpt::cie_table(), 471 * 3 * sizeof(float), (void**)&ctx->cie, scratch))) return rc;
  ctx->scene.bb = ctx->bb;
  ctx->scene.cie = ctx->cie;

  ctx->film_count = (uint64_t)cfg->output_size[0] * (uint64_t)cfg->output_size[1] * 4;
  VPT_HIP(hipMalloc((void**)&ctx->film, ctx->film_count * sizeof(float)));
  VPT_HIP(hipMemset(ctx->film, 0, ctx->film_count * sizeof(float)));
  VPT_HIP(hipMalloc((void**)&ctx->job_counter, kLaunchSlots * 2 * sizeof(unsigned long long)));  // jobs, events
  for (uint32_t i = 0; i < kLaunchSlots; ++i)
    VPT_HIP(hipEventCreateWithFlags(&ctx->slot_done[i], hipEventDisableTiming));
  VPT_HIP(hipMalloc((void**)&ctx->counters, vpt::kCounterCount * sizeof(unsigned long long)));
  VPT_HIP(hipMemset(ctx->counters, 0, vpt::kCounterCount * sizeof(unsigned long long)));
  VPT_HIP(hipMalloc((void**)&ctx->prof, kProfWords * sizeof(unsigned long long)));
  VPT_HIP(hipMemset(ctx->prof, 0, kProfWords * sizeof(unsigned long long)));
  VPT_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  VPT_HIP(hipEventCreateWithFlags(&ctx->samples_done, hipEventDisableTiming));

  // Persistent grid: as many blocks as are resident at once.
  int per_cu = 0, cus = 0;
  // sized for the production kernel of this scene; the debug variant is launched with the same grid
  VPT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, temperature ? vpt::vpt_integrate_kernel<true, false, false>
                           : (ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true> : vpt::vpt_integrate_kernel<false, false, false>),
      vpt::kBlockThreads, 0));
  VPT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  if (per_cu < 1) per_cu = 1;
  ctx->grid_blocks = per_cu * cus;
  int lat_per_cu = 0;
  VPT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &lat_per_cu, temperature ? vpt::vpt_integrate_kernel<true, false, false, true>
                               : (ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true>
                                                : vpt::vpt_integrate_kernel<false, false, false, true>),
      vpt::kBlockThreads, 0));
  ctx->lat_per_cu = std::max(1, std::min(lat_per_cu, per_cu));
  int compact_per_cu = 0;
  VPT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &compact_per_cu, temperature ? vpt::vpt_integrate_kernel<true, false, false, true, true>
                                   : (ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true, true>
                                                    : vpt::vpt_integrate_kernel<false, false, false, true, true>),
      vpt::kBlockThreads, vpt::kXchgBytes));
  ctx->compact_per_cu = compact_per_cu;
  ctx->cus = cus > 0 ? cus : 1;
  // Scheduling defaults from tools/tune.py sweeps on MI355X (C3, 256 spp): rare states run for >= 6
  // waiting lanes, density evaluations (with the deferred exact draw) for >= 36, everything runs when
  // < 8 lanes are walking; the walk loops while >= 4 lanes walk (r02 sweep: 6:8:36:4 363.7 ms vs
  // 6:12:32:4 366.6 ms, C4 103.7 vs 104.4).  The temperature kernel's rare blocks wait for 8 lanes since the film
  // regroup (C4 83.3-83.6 vs 83.9-84.3 ms over 4 alternating runs, profiles/r05gates2_c4_gate_min.txt).
  ctx->scene.gate_min = temperature ? 8 : 6;
  ctx->scene.gate_idle = 8;
  ctx->scene.gate_eval = 36;
  ctx->scene.gate_walk = 4;
  ctx->scene.pixel_mode = 0;
  ctx->scene.wave_lanes = 64;
  ctx->scene.tile_area = (uint32_t)(ctx->scene.tw * ctx->scene.th);
  VPT_HIP(hipMalloc((void**)&ctx->scene_dev, sizeof(vpt::DevScene)));
  VPT_HIP(hipMalloc((void**)&ctx->scene_lat_dev, sizeof(vpt::DevScene)));
  if ((rc = push_scene(ctx.get()))) return rc;
  lap(2);
  *out = ctx.release();
  return VPT_OK;
}

int vpt_gpu_setup_timings(const vpt_gpu_ctx* ctx, double* ms, int n) {
  if (!ctx || !ms || n < 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_setup_timings: bad argument");
  for (int i = 0; i < n && i < 5; ++i) ms[i] = ctx->setup_ms[i];
  return VPT_OK;
}

int vpt_gpu_destroy(vpt_gpu_ctx* ctx) {
  destroy(ctx);
  return VPT_OK;
}

int vpt_gpu_job_space(const vpt_gpu_ctx* ctx, uint64_t* jobs_per_wave, uint64_t* total_jobs) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (jobs_per_wave) *jobs_per_wave = ctx->scene.T;
  if (total_jobs) *total_jobs = ctx->scene.T * (uint64_t)ctx->cfg.num_waves;
  return VPT_OK;
}

int vpt_gpu_render_jobs(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film_device,
                        void* hip_stream) {
  return render(ctx, jid_begin, jid_count, film_device, nullptr, hip_stream);
}

int vpt_gpu_render_jobs_records(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film_device,
                                float* records_device, void* hip_stream) {
  return render(ctx, jid_begin, jid_count, film_device, records_device, hip_stream);
}

int vpt_gpu_trace_jobs(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film_device,
                       vpt_event* events_device, uint64_t capacity, uint64_t* count, void* hip_stream) {
  if (!ctx || !events_device || !count) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_trace_jobs: null argument");
  *count = 0;
  uint32_t slot = 0;
  int rc = render(ctx, jid_begin, jid_count, film_device, nullptr, hip_stream, events_device, capacity, &slot);
  if (rc) return rc;
  if (jid_count == 0) return VPT_OK;
  unsigned long long n = 0;
  VPT_HIP(hipMemcpyAsync(&n, ctx->job_counter + 2 * slot + 1, sizeof n, hipMemcpyDeviceToHost, (hipStream_t)hip_stream));
  VPT_HIP(hipStreamSynchronize((hipStream_t)hip_stream));
  *count = n;
  return VPT_OK;
}

int vpt_gpu_majorant_trace(vpt_gpu_ctx* ctx, const float origin[3], const float direction[3], float* rows_host,
                           int max_rows, int* n_rows) {
  if (!ctx || !origin || !direction || !n_rows || (max_rows > 0 && !rows_host) || max_rows < 0)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_majorant_trace: bad argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  float* rows = nullptr;
  int* n = nullptr;
  VPT_HIP(hipMalloc((void**)&rows, (size_t)(max_rows > 0 ? max_rows : 1) * 9 * sizeof(float)));
  if (hipMalloc((void**)&n, sizeof(int)) != hipSuccess) {
    (void)hipFree(rows);
    return vpt::set_error(VPT_E_HIP, "vpt_gpu_majorant_trace: hipMalloc failed");
  }
  hipLaunchKernelGGL(vpt::vpt_majorant_trace_kernel, dim3(1), dim3(64), 0, nullptr, ctx->scene_dev, origin[0],
                     origin[1], origin[2], direction[0], direction[1], direction[2], rows, max_rows, n);
  hipError_t e = hipGetLastError();
  int nn = 0;
  if (e == hipSuccess) e = hipMemcpy(&nn, n, sizeof nn, hipMemcpyDeviceToHost);
  if (e == hipSuccess && max_rows > 0)
    e = hipMemcpy(rows_host, rows, (size_t)std::min(nn, max_rows) * 9 * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(rows);
  (void)hipFree(n);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_majorant_trace: ") + hipGetErrorString(e));
  *n_rows = nn;
  return VPT_OK;
}

int vpt_gpu_set_rng_mode(vpt_gpu_ctx* ctx, int mode) {
  if (!ctx || (mode != VPT_RNG_REFERENCE && mode != VPT_RNG_PIXEL))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_rng_mode: bad argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if (mode == VPT_RNG_PIXEL && (int64_t)ctx->scene.tw * ctx->scene.th >= (int64_t)vpt::kPixelTaken)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_rng_mode: tile too large for the pixel mode");
  ctx->scene.pixel_mode = mode == VPT_RNG_PIXEL ? 1 : 0;
  ctx->scene.tile_area = (uint32_t)(ctx->scene.tw * ctx->scene.th);
  return push_scene(ctx);
}

int vpt_gpu_set_pixel_chunk(vpt_gpu_ctx* ctx, int chunk) {
  if (!ctx || chunk < 0 || (chunk & (chunk - 1)) != 0 || (chunk > 0 && ctx->scene.tile_area % (uint32_t)chunk != 0))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_pixel_chunk: 0 or a power of two dividing the tile area");
  ctx->pixel_chunk = chunk;  // read by the next render's host code only: no wait
  return VPT_OK;
}

int vpt_gpu_set_run_skipping(vpt_gpu_ctx* ctx, int mode) {
  if (!ctx || mode < -1 || mode > 1) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_run_skipping: bad argument");
  if (mode == 1 && ctx->scene.has_temperature)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_run_skipping: no run-skipping variant with a temperature grid");
  ctx->use_runs = mode < 0 ? (!ctx->scene.has_temperature && ctx->density.run_fraction >= 0.25) : mode == 1;
  return VPT_OK;
}

int vpt_gpu_kernel_variant(const vpt_gpu_ctx* ctx, int* has_temperature, int* run_skipping) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (has_temperature) *has_temperature = ctx->scene.has_temperature ? 1 : 0;
  if (run_skipping) *run_skipping = ctx->use_runs ? 1 : 0;
  return VPT_OK;
}

int vpt_gpu_set_film_order(vpt_gpu_ctx* ctx, int mode, uint64_t max_bytes) {
  if (!ctx || (mode != VPT_FILM_ATOMIC && mode != VPT_FILM_ORDERED))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_film_order: bad argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  ctx->film_order = mode;
  ctx->film_order_max = max_bytes;
  if (mode == VPT_FILM_ATOMIC && ctx->samples && ctx->open_feeds.load() == 0) {  // the buffer is not needed
    if (ctx->samples_used) VPT_HIP(hipEventSynchronize(ctx->samples_done));
    (void)hipFree(ctx->samples);
    ctx->samples = nullptr;
    ctx->samples_bytes = 0;
  }
  return VPT_OK;
}

int vpt_gpu_film_order_info(const vpt_gpu_ctx* ctx, int* mode, uint64_t* buffer_bytes, uint64_t* ordered_launches,
                            uint64_t* atomic_launches) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (mode) *mode = ctx->film_order;
  if (buffer_bytes) *buffer_bytes = ctx->samples_bytes;
  if (ordered_launches) *ordered_launches = ctx->ordered_launches;
  if (atomic_launches) *atomic_launches = ctx->atomic_launches;
  return VPT_OK;
}

int vpt_gpu_set_job_order(vpt_gpu_ctx* ctx, int mode) {
  if (!ctx || mode < VPT_ORDER_JID || mode > VPT_ORDER_COST_TAIL)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_order: bad argument");
  ctx->order_mode = mode;
  return VPT_OK;
}

int vpt_gpu_set_job_order_tail(vpt_gpu_ctx* ctx, int waves) {
  if (!ctx || waves < 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_order_tail: bad argument");
  ctx->order_tail_waves = waves;
  return VPT_OK;
}

int vpt_gpu_tile_costs(vpt_gpu_ctx* ctx, float* cost, uint32_t* rank) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = ensure_order(ctx))) return rc;
  if (cost) std::memcpy(cost, ctx->tile_cost.data(), ctx->tile_cost.size() * sizeof(float));
  if (rank) std::memcpy(rank, ctx->tile_rank.data(), ctx->tile_rank.size() * sizeof(uint32_t));
  return VPT_OK;
}

int vpt_gpu_set_tile_costs(vpt_gpu_ctx* ctx, const float* cost) {
  if (!ctx || !cost) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_tile_costs: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  for (uint64_t i = 0; i < ctx->scene.T; ++i)  // NaN would break the sort's strict weak ordering
    if (!std::isfinite(cost[i])) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_tile_costs: non-finite cost");
  if ((rc = wait_ctx(ctx))) return rc;  // in-flight launches read the current order
  ctx->tile_cost.assign(cost, cost + ctx->scene.T);
  return rank_tiles(ctx);
}

int vpt_gpu_set_job_permutation(vpt_gpu_ctx* ctx, const uint32_t* perm, uint64_t n) {
  if (!ctx || (n && !perm)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_permutation: null argument");
  if (n >= (1ULL << 32)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_permutation: too many jobs");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  std::vector<uint8_t> seen(n, 0);
  for (uint64_t i = 0; i < n; ++i) {
    if (perm[i] >= n || seen[perm[i]]) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_permutation: not a permutation");
    seen[perm[i]] = 1;
  }
  if ((rc = wait_ctx(ctx))) return rc;  // in-flight launches may read the current one
  (void)hipFree(ctx->perm);
  ctx->perm = nullptr;
  ctx->perm_n = 0;
  if (n == 0) return VPT_OK;
  VPT_HIP(hipMalloc((void**)&ctx->perm, n * sizeof(uint32_t)));
  VPT_HIP(hipMemcpy(ctx->perm, perm, n * sizeof(uint32_t), hipMemcpyHostToDevice));
  ctx->perm_n = n;
  return VPT_OK;
}

int vpt_gpu_sync(vpt_gpu_ctx* ctx) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  return wait_ctx(ctx);
}

int vpt_gpu_stream_create(vpt_gpu_ctx* ctx, void** hip_stream) {
  if (!ctx || !hip_stream) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_stream_create: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  hipStream_t s = nullptr;
  VPT_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *hip_stream = s;
  return VPT_OK;
}

int vpt_gpu_bind_thread_near(vpt_gpu_ctx* ctx, int* node_out) {
  if (node_out) *node_out = -1;
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_bind_thread_near: null context");
  char bus[64] = {};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, ctx->device) != hipSuccess) return VPT_OK;
  for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
  int node = -1;
  {
    std::ifstream in(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
    if (!(in >> node) || node < 0) return VPT_OK;
  }
  std::ifstream in("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(in, list)) return VPT_OK;
  // Allowed: the process's CPUs (its main thread's set: taskset / numactl restrict it), not this thread's own --
  // a thread inherits its creator's set, and a caller bound to the far node would otherwise pin its helpers
  // there too (r05n: a taker on node 1 made the pusher it started run there).
  cpu_set_t cur, near;
  CPU_ZERO(&near);
  if (sched_getaffinity(getpid(), sizeof cur, &cur) != 0) return VPT_OK;
  // "0-63,128-191"
  for (size_t pos = 0; pos < list.size();) {
    size_t end = list.find(',', pos);
    if (end == std::string::npos) end = list.size();
    const std::string r = list.substr(pos, end - pos);
    const size_t dash = r.find('-');
    const int a = std::atoi(r.c_str()), b = dash == std::string::npos ? a : std::atoi(r.c_str() + dash + 1);
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (c >= 0 && CPU_ISSET(c, &cur)) CPU_SET(c, &near);
    pos = end + 1;
  }
  if (CPU_COUNT(&near) == 0) return VPT_OK;
  if (pthread_setaffinity_np(pthread_self(), sizeof near, &near) != 0) return VPT_OK;
  if (node_out) *node_out = node;
  return VPT_OK;
}

int vpt_gpu_stream_destroy(vpt_gpu_ctx* ctx, void* hip_stream) {
  if (!ctx || !hip_stream) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_stream_destroy: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  VPT_HIP(hipStreamDestroy((hipStream_t)hip_stream));
  return VPT_OK;
}

int vpt_gpu_stream_sync(vpt_gpu_ctx* ctx, void* hip_stream) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_stream_sync: null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  VPT_HIP(hipStreamSynchronize((hipStream_t)hip_stream));
  return VPT_OK;
}

int vpt_gpu_film_alloc(vpt_gpu_ctx* ctx, float** film_device) {
  if (!ctx || !film_device) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_film_alloc: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  float* f = nullptr;
  VPT_HIP(hipMalloc((void**)&f, ctx->film_count * sizeof(float)));
  const hipError_t e = hipMemset(f, 0, ctx->film_count * sizeof(float));
  if (e != hipSuccess) {
    (void)hipFree(f);
    return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_film_alloc: ") + hipGetErrorString(e));
  }
  *film_device = f;
  return VPT_OK;
}

int vpt_gpu_film_free(vpt_gpu_ctx* ctx, float* film_device) {
  if (!ctx || !film_device || film_device == ctx->film)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_film_free: not a film from vpt_gpu_film_alloc");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  VPT_HIP(hipFree(film_device));
  return VPT_OK;
}

int vpt_gpu_film_flush_to_host(vpt_gpu_ctx* ctx, float* film_device, float* film_host) {
  if (!ctx || !film_host) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_film_flush_to_host: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  float* f = film_device ? film_device : ctx->film;
  const size_t bytes = ctx->film_count * sizeof(float);
  if (!ctx->staging) VPT_HIP(hipHostMalloc((void**)&ctx->staging, bytes, hipHostMallocDefault));
  VPT_HIP(hipMemcpyAsync(ctx->staging, f, bytes, hipMemcpyDeviceToHost, ctx->stream));
  VPT_HIP(hipMemsetAsync(f, 0, bytes, ctx->stream));
  VPT_HIP(hipStreamSynchronize(ctx->stream));
  const float* src = ctx->staging;
  for (uint64_t i = 0; i < ctx->film_count; ++i) film_host[i] += src[i];
  return VPT_OK;
}

}  // extern "C"

// A feed: one launch of the production kernel that renders job ids as the host pushes them (see
// include/vpt_gpu.h).  Its host-pinned, coherent block holds the published word, the error word and the
// started hint, then the ring of job ids, then the per-tile job counts pushed.
struct vpt_gpu_feed {
  vpt_gpu_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;
  float* film = nullptr;
  uint64_t* block = nullptr;  // hipHostMalloc'd: [8] word, error word, waiting word, padding, [4..8) the started
                              // hints; [cap] ring; uint32 counts[T]
  uint64_t* word = nullptr;
  uint32_t* error = nullptr;    // block[1]: a lane that gave up waiting stores 1 here
  uint64_t* started = nullptr;  // block[4..4 + kHintSlots): reported reserved items (kStartedHint)
  uint64_t* waiting = nullptr;  // block[2]: the job count a wavefront saw when it ran out of published items
  uint64_t* ring = nullptr;
  uint32_t* counts = nullptr;
  bool stage = false;
  // Staged feeds: the launch counts the jobs it completes per tile in device memory; snapshots and the final
  // collect copy that and the film into pinned memory with the copy engines (beside the launch, which holds
  // every CU) and add what is new since the previous copy into the caller's film.
  uint32_t* done_dev = nullptr;   // uint32[T]
  float* pin_film = nullptr;      // film_count floats, pinned
  uint32_t* pin_done = nullptr;   // uint32[T], pinned
  std::vector<float> shown;       // the film as already added to the caller's film
  std::vector<uint32_t> shown_done;
  hipStream_t copy_stream = nullptr;
  hipStream_t own_stream = nullptr;  // a staged feed's launch stream when the caller passes none
  bool ring_clean = false;           // every slot holds kFeedEmpty (a completed feed's lanes marked them all)
  uint64_t cap = 0;
  uint64_t published = 0;
  uint64_t started_seen = 0;
  std::chrono::steady_clock::time_point started_moved{};  // when started_seen last moved (vpt_gpu_feed_backlog)
  std::chrono::steady_clock::time_point stale_traced{};
  hipEvent_t closed_ev = nullptr;
  bool closed = false;
  bool launched = false;     // the launch starts once launch_at items are published, or at close
  bool counted = false;      // counted in ctx->open_feeds (launched, not closed)
  uint64_t launch_at = 0;
  vpt::FeedLaunch fl{};
};

namespace {
constexpr double kFeedHostWaitS = 120.0;  // a push waiting this long for a ring slot gives up
constexpr size_t kZeroBytes = 4u << 20;   // the context's pinned zeros (staged feeds' clears)

// VPT_FEED_TRACE=1: one stderr line per feed event (open / launch / close / a push's wait for a ring slot /
// snapshots / the end of its work), milliseconds since the first event -- for diagnosing a drop-in's protocol.
void feed_trace(const vpt_gpu_feed* f, const char* what, double a = 0, double b = 0) {
  static const bool on = std::getenv("VPT_FEED_TRACE") && std::atoi(std::getenv("VPT_FEED_TRACE")) > 0;
  if (!on) return;
  static const auto t0 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "feed %10.2f ms %p %-8s %.0f %.0f\n", ms, (const void*)f, what, a, b);
}

void feed_free(vpt_gpu_feed* f) {
  if (!f) return;
  (void)hipSetDevice(f->ctx->device);
  if (f->closed_ev) (void)hipEventDestroy(f->closed_ev);
  if (f->copy_stream) (void)hipStreamDestroy(f->copy_stream);
  if (f->own_stream) (void)hipStreamDestroy(f->own_stream);
  (void)hipHostFree(f->block);
  if (f->pin_film) (void)hipHostFree(f->pin_film);
  if (f->pin_done) (void)hipHostFree(f->pin_done);
  (void)hipFree(f->done_dev);
  delete f;
}

void feed_pool_free(vpt_gpu_ctx* ctx) {
  for (vpt_gpu_feed* f : ctx->feed_pool) feed_free(f);
  ctx->feed_pool.clear();
  if (ctx->zeros) (void)hipHostFree(ctx->zeros);
  ctx->zeros = nullptr;
}

// Publishes items [0, published) and, with close, the end of the feed (release: the ring and count
// stores are visible to the GPU before the word that publishes them).
void feed_publish(vpt_gpu_feed* f, bool close) {
  __atomic_store_n(f->word, f->published | (close ? vpt::kFeedClosed : 0), __ATOMIC_RELEASE);
}

// Zeroes `bytes` of device memory with host-to-device copies of the context's pinned zeros, enqueued on s:
// copy-engine work, which runs while another launch holds every CU (a fill kernel would wait for it).
int clear_by_copy(vpt_gpu_ctx* ctx, void* dev, size_t bytes, hipStream_t s) {
  if (!ctx->zeros) {
    VPT_HIP(hipHostMalloc((void**)&ctx->zeros, kZeroBytes, hipHostMallocDefault));
    std::memset(ctx->zeros, 0, kZeroBytes);
  }
  for (size_t off = 0; off < bytes; off += kZeroBytes)
    VPT_HIP(hipMemcpyAsync(static_cast<char*>(dev) + off, ctx->zeros, std::min(kZeroBytes, bytes - off),
                           hipMemcpyHostToDevice, s));
  return VPT_OK;
}

// The resources of a feed of ring size cap (and, staged, its copy-out buffers), from the context's pool or new.
int feed_get(vpt_gpu_ctx* ctx, uint64_t cap, bool stage, std::unique_ptr<vpt_gpu_feed, void (*)(vpt_gpu_feed*)>& f) {
  for (size_t i = 0; i < ctx->feed_pool.size(); ++i)
    if (ctx->feed_pool[i]->cap == cap && (!stage || ctx->feed_pool[i]->done_dev)) {  // a pooled feed of this window
      f.reset(ctx->feed_pool[i]);
      ctx->feed_pool.erase(ctx->feed_pool.begin() + (ptrdiff_t)i);
      return VPT_OK;
    }
  f.reset(new vpt_gpu_feed());
  f->ctx = ctx;
  f->cap = cap;
  const uint64_t T = ctx->scene.T;
  const size_t bytes = (vpt::kFeedHeaderWords + cap) * sizeof(uint64_t) + T * sizeof(uint32_t);
  VPT_HIP(hipHostMalloc((void**)&f->block, bytes, hipHostMallocCoherent | hipHostMallocMapped));
  f->word = f->block;
  f->error = reinterpret_cast<uint32_t*>(f->block + 1);
  f->started = f->block + 4;
  f->waiting = f->block + 2;
  f->ring = f->block + vpt::kFeedHeaderWords;
  f->counts = reinterpret_cast<uint32_t*>(f->ring + cap);
  VPT_HIP(hipEventCreateWithFlags(&f->closed_ev, hipEventDisableTiming));
  if (stage) {
    VPT_HIP(hipMalloc((void**)&f->done_dev, T * sizeof(uint32_t)));
    VPT_HIP(hipHostMalloc((void**)&f->pin_film, ctx->film_count * sizeof(float), hipHostMallocDefault));
    VPT_HIP(hipHostMalloc((void**)&f->pin_done, T * sizeof(uint32_t), hipHostMallocDefault));
    VPT_HIP(hipStreamCreateWithFlags(&f->copy_stream, hipStreamNonBlocking));
    VPT_HIP(hipStreamCreateWithFlags(&f->own_stream, hipStreamNonBlocking));
    f->shown.assign(ctx->film_count, 0.0f);
    f->shown_done.assign(T, 0u);
    if (int rc = clear_by_copy(ctx, f->done_dev, T * sizeof(uint32_t), f->copy_stream)) return rc;
    VPT_HIP(hipStreamSynchronize(f->copy_stream));
  }
  return VPT_OK;
}

uint64_t feed_cap(const vpt_gpu_ctx* ctx, uint64_t window) {
  // The ring holds at least twice the launch's lanes: a lane reserves an item only while some are
  // published, so reservations lead the consumed items by at most the lanes, and the host keeps pushing
  // while the lanes it has already fed work (C3: 458 752 lanes, ring 2^20).
  const uint64_t lanes = (uint64_t)ctx->grid_blocks * vpt::kBlockThreads;
  uint64_t cap = 1024;
  while ((cap < window || cap < 2 * lanes) && cap < (1ULL << 26)) cap <<= 1;
  return cap;
}
}  // namespace

namespace {
int feed_open(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window, bool stage, vpt_gpu_feed** out) {
  if (!ctx || !out || (!hip_stream && !stage)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_open: null argument");
  *out = nullptr;
  if (ctx->scene.pixel_mode) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_open: feeds run the reference RNG mode");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  const uint64_t cap = feed_cap(ctx, window);
  std::unique_ptr<vpt_gpu_feed, void (*)(vpt_gpu_feed*)> f(nullptr, feed_free);
  if ((rc = feed_get(ctx, cap, stage, f))) return rc;
  f->stage = stage;
  f->stream = hip_stream ? (hipStream_t)hip_stream : f->own_stream;  // (staged: the feed's own stream if none)
  f->film = film_device ? film_device : ctx->film;
  f->published = 0;
  f->started_seen = 0;
  f->started_moved = {};
  f->closed = false;
  f->counted = false;
  if (!f->ring_clean)
    for (uint64_t i = 0; i < cap; ++i) f->ring[i] = vpt::kFeedEmpty;
  f->ring_clean = false;
  std::memset(f->counts, 0, ctx->scene.T * sizeof(uint32_t));
  __atomic_store_n(f->error, 0u, __ATOMIC_RELAXED);
  for (uint64_t i = 0; i < vpt::kHintSlots; ++i) __atomic_store_n(f->started + i, 0ULL, __ATOMIC_RELAXED);
  __atomic_store_n(f->waiting, 0ULL, __ATOMIC_RELAXED);
  __atomic_store_n(f->word, 0ULL, __ATOMIC_RELEASE);
  uint64_t* word_dev = nullptr;
  VPT_HIP(hipHostGetDevicePointer((void**)&word_dev, f->word, 0));
  f->fl = vpt::FeedLaunch{word_dev, word_dev + vpt::kFeedHeaderWords, cap - 1, reinterpret_cast<unsigned*>(word_dev + 1),
                          word_dev + 4, word_dev + 2,
                          stage ? f->done_dev : nullptr};
  // The launch is deferred until the ring holds as many items as it has lanes (or the feed is closed):
  // launched at once, its idle wavefronts would poll the host link for work (r04).
  f->launched = false;
  f->launch_at = (uint64_t)ctx->grid_blocks * vpt::kBlockThreads;
  // (With the urgent-fetch gate, launching at 1/4 or 1/16 of the lanes no longer stalls, but gains nothing
  // measurable either: C3 368.6-372.7 vs 368.4-376.2 ms, C4 116-137 vs 117-134; r05u2.)
  // (Launching at a quarter or a sixteenth of the lanes saved nothing and stalled: lanes racing past the
  // published count hold items their waves serve late, and the wrapping ring waits for them; r05k.)
  feed_trace(f.get(), stage ? "open_stg" : "open", (double)cap, (double)(uintptr_t)hip_stream);
  *out = f.release();
  return VPT_OK;
}

int feed_launch(vpt_gpu_feed* f) {
  if (f->launched) return VPT_OK;
  f->launched = true;
  if (!f->closed) {  // launched and open: it holds the device until it is closed
    ++f->ctx->open_feeds;
    f->counted = true;
  }
  feed_trace(f, "launch", (double)f->published);
  return render(f->ctx, 0, ~0ULL >> 1, f->film, nullptr, f->stream, nullptr, 0, nullptr, &f->fl);
}

// film_host += (the staged feed's film and per-tile counts as copied to pin_film / pin_done) - (what was added
// before), rows split over a few threads; shown := the copy.  Counts are integers (exact); the radiance
// channels telescope to the final film (the first add onto zero is exact).
void add_delta(vpt_gpu_feed* f, float* film_host) {
  const vpt::DevScene& S = f->ctx->scene;
  const uint64_t T = S.T;
  std::vector<uint32_t> dc(T);
  for (uint64_t t = 0; t < T; ++t) {
    // (a copy taken beside the launch reads memory, not the dirty L2 lines: it may lag, never lead; the max
    // keeps the counts monotone should an older value be read after a newer one)
    const uint32_t now = std::max(f->pin_done[t], f->shown_done[t]);
    dc[t] = now - f->shown_done[t];
    f->shown_done[t] = now;
  }
  auto rows = [&](int32_t y0, int32_t y1) {
    for (int32_t y = y0; y < y1; ++y) {
      const uint32_t* dct = dc.data() + (uint64_t)(y / S.th) * S.ntx;
      for (int32_t x = 0; x < S.W; ++x) {
        const uint64_t p = ((uint64_t)y * (uint64_t)S.W + (uint64_t)x) * 4;
        const bool counted = !S.single_pixel_enabled || (x == S.sp_x && y == S.sp_y);
        for (int c = 0; c < 3; ++c) {
          const float v = f->pin_film[p + c];
          film_host[p + c] += v - f->shown[p + c];
          f->shown[p + c] = v;
        }
        if (counted) film_host[p + 3] += (float)dct[x / S.tw];
      }
    }
  };
  const int32_t H = S.H;
  const unsigned hw = std::thread::hardware_concurrency();
  const int nt = (int)std::max(1u, std::min(8u, hw ? hw : 1u));
  if (nt == 1 || (uint64_t)S.W * (uint64_t)H < (1u << 16)) {
    rows(0, H);
    return;
  }
  std::vector<std::thread> pool;
  for (int i = 1; i < nt; ++i) pool.emplace_back(rows, (int32_t)((int64_t)H * i / nt), (int32_t)((int64_t)H * (i + 1) / nt));
  rows(0, (int32_t)((int64_t)H / nt));
  for (auto& t : pool) t.join();
}

// Copies a staged feed's film and per-tile counts with the copy engines and adds what is new into film_host.
// after_end: ordered after the feed's launch (exact); else beside it (what it has completed so far).
int feed_snapshot(vpt_gpu_feed* f, float* film_host, bool after_end, const std::function<int()>& then = {}) {
  vpt_gpu_ctx* ctx = f->ctx;
  if (after_end) VPT_HIP(hipStreamWaitEvent(f->copy_stream, f->closed_ev, 0));
  // counts first: a job counted here has added its samples before (in its lane's order)
  feed_trace(f, after_end ? "final0" : "snap0");
  VPT_HIP(hipMemcpyAsync(f->pin_done, f->done_dev, ctx->scene.T * sizeof(uint32_t), hipMemcpyDeviceToHost, f->copy_stream));
  VPT_HIP(hipMemcpyAsync(f->pin_film, f->film, ctx->film_count * sizeof(float), hipMemcpyDeviceToHost, f->copy_stream));
  hipEvent_t copied = nullptr;
  VPT_HIP(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
  hipError_t e = hipEventRecord(copied, f->copy_stream);
  int rc = VPT_OK;
  if (e == hipSuccess && then) rc = then();  // queued after the copy: runs while the host adds it
  if (e == hipSuccess) e = hipEventSynchronize(copied);
  (void)hipEventDestroy(copied);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("feed snapshot copy: ") + hipGetErrorString(e));
  if (rc) return rc;
  feed_trace(f, "copied");
  add_delta(f, film_host);
  feed_trace(f, after_end ? "final" : "snapshot");
  return VPT_OK;
}

// Waits for a closed feed's work; a staged feed then adds its film into film_host (when given) and clears its
// film and counts for the next use.  The feed goes back to the context's pool unless a HIP failure leaves its
// launch possibly still reading the block (then it leaks).
int feed_finish(vpt_gpu_feed* f, float* film_host) {
  bool complete = false;
  int rc = VPT_OK;
  feed_trace(f, "wait", (double)f->published);
  const hipError_t e = hipEventSynchronize(f->closed_ev);
  if (e != hipSuccess)
    rc = vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_feed_destroy: ") + hipGetErrorString(e));
  else
    complete = true;
  feed_trace(f, "ended", (double)f->published, complete ? (double)__atomic_load_n(f->error, __ATOMIC_ACQUIRE) : -1.0);
  if (complete && __atomic_load_n(f->error, __ATOMIC_ACQUIRE))
    rc = vpt::set_error(VPT_E_STATE, "vpt_gpu_feed_destroy: lanes of the feed's launch gave up waiting for jobs");
  if (complete && f->stage) {
    vpt_gpu_ctx* ctx = f->ctx;
    // the final copy; then the film and counts back to zero (copy engines, queued behind the copy on the same
    // stream) while the host adds the copy; nothing shown afterwards
    auto clear = [&] {
      int r = clear_by_copy(ctx, f->film, ctx->film_count * sizeof(float), f->copy_stream);
      return r ? r : clear_by_copy(ctx, f->done_dev, ctx->scene.T * sizeof(uint32_t), f->copy_stream);
    };
    if (rc == VPT_OK && film_host) {
      rc = feed_snapshot(f, film_host, true, clear);
    } else {
      const int r = clear();
      if (rc == VPT_OK) rc = r;
    }
    if (hipStreamSynchronize(f->copy_stream) != hipSuccess && rc == VPT_OK)
      rc = vpt::set_error(VPT_E_HIP, "vpt_gpu_feed_collect: clearing the film failed");
    std::fill(f->shown.begin(), f->shown.end(), 0.0f);
    std::fill(f->shown_done.begin(), f->shown_done.end(), 0u);
    feed_trace(f, "cleared");
  }
  // a completed feed's lanes marked every published slot empty (unpublished ones still are)
  f->ring_clean = complete && rc == VPT_OK;
  if (complete) f->ctx->feed_pool.push_back(f);
  return rc;
}
}  // namespace

extern "C" {

int vpt_gpu_feed_open(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window, vpt_gpu_feed** out) {
  return feed_open(ctx, film_device, hip_stream, window, false, out);
}

int vpt_gpu_feed_open_staged(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window,
                             vpt_gpu_feed** out) {
  return feed_open(ctx, film_device, hip_stream, window, true, out);
}

int vpt_gpu_feed_prepare(vpt_gpu_ctx* ctx, uint64_t window, int staged) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_prepare: null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  std::unique_ptr<vpt_gpu_feed, void (*)(vpt_gpu_feed*)> f(nullptr, feed_free);
  if ((rc = feed_get(ctx, feed_cap(ctx, window), staged != 0, f))) return rc;
  if (staged && (rc = clear_by_copy(ctx, ctx->zeros, 0, f->copy_stream))) return rc;  // (allocates the zeros)
  ctx->feed_pool.push_back(f.release());
  return VPT_OK;
}

int vpt_gpu_feed_push(vpt_gpu_feed* f, const uint64_t* jids, uint64_t n) {
  if (!f || (n && !jids)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_push: null argument");
  if (f->closed) return vpt::set_error(VPT_E_STATE, "vpt_gpu_feed_push: the feed is closed");
  const uint64_t T = f->ctx->scene.T, mask = f->cap - 1;
  const bool count = !f->stage;  // (a staged feed's launch counts its completed jobs itself)
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t jid = jids[i];
    if (jid >> 62) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_push: job id out of range");
    // The ring's lines were last written by the lanes (their empty marks): each is a miss in the host's
    // caches, so they are fetched 32 lines ahead (r05: the pusher, not the provider, bounded C4's drain).
    if ((f->published & 7) == 0) __builtin_prefetch(f->ring + ((f->published + 256) & mask), 1);
    uint64_t* slot = f->ring + (f->published & mask);
    if (__atomic_load_n(slot, __ATOMIC_ACQUIRE) != vpt::kFeedEmpty) {
      // the window is full (cap items published and not yet started): publish what we have, then wait --
      // spinning first (slots free at the GPU's job rate, tens of millions a second: a sleep between
      // checks would hold the lanes back), sleeping once the wait is long (a launch not yet started).  The
      // limit counts from the start of this wait, not of the call.
      feed_publish(f, false);
      if (int rc = feed_launch(f)) return rc;
      const auto w0 = std::chrono::steady_clock::now();
      for (uint32_t spins = 0; __atomic_load_n(slot, __ATOMIC_ACQUIRE) != vpt::kFeedEmpty; ++spins) {
        if (spins < (1u << 16)) continue;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count() > kFeedHostWaitS)
          return vpt::set_error(VPT_E_STATE, "vpt_gpu_feed_push: the feed's launch stopped taking jobs");
      }
      const double waited = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
      if (waited > 1.0) feed_trace(f, "slotwait", (double)f->published, waited);
    }
    *slot = jid;
    if (count) ++f->counts[jid % T];
    ++f->published;
  }
  feed_publish(f, false);
  if (f->published >= f->launch_at)
    if (int rc = feed_launch(f)) return rc;
  return VPT_OK;
}

constexpr std::chrono::milliseconds kStaleHints{10};

int vpt_gpu_feed_backlog(vpt_gpu_feed* f, uint64_t* backlog) {
  if (!f || !backlog) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_backlog: null argument");
  // the newest reported reservation (the lanes' posted writes may land out of order: keep the largest)
  uint64_t s = 0;  // the largest reported reservation (each slot only grows between two of its writes)
  for (uint64_t i = 0; i < vpt::kHintSlots; ++i) s = std::max(s, __atomic_load_n(f->started + i, __ATOMIC_RELAXED));
  const auto now = std::chrono::steady_clock::now();
  if (s > f->started_seen || f->started_moved == std::chrono::steady_clock::time_point{}) {
    f->started_seen = std::max(s, f->started_seen);
    f->started_moved = f->stale_traced = now;
  }
  *backlog = f->published > f->started_seen ? f->published - f->started_seen : 0;
  // The hints may land out of order, so the estimate can read high after a burst of reservations (a launch's
  // first lane's worth reserves within microseconds) -- and with no reservation after it to correct it, a
  // pusher waiting for that backlog to drain would wait for ever while the lanes wait for it (r05q).  A
  // wavefront that runs out of published items stores the job count it saw: one >= the published count means
  // the lanes are waiting now.
  const uint64_t waiting = __atomic_load_n(f->waiting, __ATOMIC_RELAXED);
  if (f->launched && waiting >= f->published) *backlog = 0;
  // And a host-side bound: hints that have not moved for kStaleHints while the estimate says jobs
  // are queued mean either lanes too busy to take any -- pushing more only fills the ring up to its window --
  // or an estimate stuck on a stale count: read it as empty, so the pusher never waits on it for long.
  if (f->launched && *backlog > 0 && now - f->started_moved > kStaleHints) *backlog = 0;
  if (f->launched && *backlog > 0 && now - f->started_moved > std::chrono::seconds(1) &&
      now - f->stale_traced > std::chrono::seconds(1)) {  // (diagnostics) nothing reserved for a second
    f->stale_traced = now;
    const hipError_t q = hipStreamQuery(f->stream);
    feed_trace(f, "noreserve", (double)f->published, (double)f->started_seen);
    feed_trace(f, "state", (double)__atomic_load_n(f->error, __ATOMIC_RELAXED),
               q == hipSuccess ? 1.0 : (q == hipErrorNotReady ? 0.0 : -(double)q));
  }
  return VPT_OK;
}

int vpt_gpu_feed_debug(vpt_gpu_feed* f, int op, uint64_t* value) {
  if (!f || !value || op < 0 || op > 2) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_debug: bad argument");
  if (op == 0) {
    *value = __atomic_load_n(f->waiting, __ATOMIC_RELAXED);
  } else if (op == 1) {
    __atomic_store_n(f->waiting, *value, __ATOMIC_RELAXED);
  } else {
    for (uint64_t i = 0; i < vpt::kHintSlots; ++i) __atomic_store_n(f->started + i, *value, __ATOMIC_RELAXED);
    f->started_seen = *value;
  }
  return VPT_OK;
}

int vpt_gpu_feed_close(vpt_gpu_feed* f) {
  if (!f) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_close: null feed");
  if (f->closed) return VPT_OK;
  int rc = ctx_device(f->ctx);
  if (rc) return rc;
  f->closed = true;
  feed_publish(f, true);
  feed_trace(f, "close", (double)f->published);
  rc = feed_launch(f);
  if (f->counted) {  // closed: its launch ends once its jobs are done
    --f->ctx->open_feeds;
    f->counted = false;
  }
  if (rc) return rc;
  if (f->stage) {  // the host adds the film and the counts at collect (copy engines)
    VPT_HIP(hipEventRecord(f->closed_ev, f->stream));
    return VPT_OK;
  }
  // after the launch: the pushed jobs' sample counts (read from the pinned block, final now)
  uint32_t* counts_dev = nullptr;
  VPT_HIP(hipHostGetDevicePointer((void**)&counts_dev, f->counts, 0));
  const uint64_t npix = (uint64_t)f->ctx->scene.W * (uint64_t)f->ctx->scene.H;
  hipLaunchKernelGGL(vpt::vpt_tile_count_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, f->stream,
                     f->ctx->scene_dev, f->film, counts_dev);
  VPT_HIP(hipGetLastError());
  VPT_HIP(hipEventRecord(f->closed_ev, f->stream));
  return VPT_OK;
}

int vpt_gpu_feed_query(vpt_gpu_feed* f, int* done, uint64_t* pushed) {
  if (!f) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_query: null feed");
  if (pushed) *pushed = f->published;
  if (done) {
    *done = 0;
    if (f->closed) {
      const hipError_t e = hipEventQuery(f->closed_ev);
      if (e == hipSuccess)
        *done = 1;
      else if (e != hipErrorNotReady)
        return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_feed_query: ") + hipGetErrorString(e));
    }
  }
  return VPT_OK;
}

int vpt_gpu_feed_destroy(vpt_gpu_feed* f) {
  if (!f) return VPT_OK;
  const int rc = vpt_gpu_feed_close(f);
  return rc ? rc : feed_finish(f, nullptr);
}

int vpt_gpu_feed_snapshot(vpt_gpu_feed* f, float* film_host) {
  if (!f || !film_host) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_snapshot: null argument");
  if (!f->stage) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_snapshot: not a staged feed (vpt_gpu_feed_open_staged)");
  int rc = ctx_device(f->ctx);
  if (rc) return rc;
  return feed_snapshot(f, film_host, false);
}

int vpt_gpu_feed_collect(vpt_gpu_feed* f, float* film_host) {
  if (!f || !film_host) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_collect: null argument");
  if (!f->stage) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_collect: not a staged feed (vpt_gpu_feed_open_staged)");
  const int rc = vpt_gpu_feed_close(f);
  return rc ? rc : feed_finish(f, film_host);
}

int vpt_gpu_film_clear(vpt_gpu_ctx* ctx) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;  // renders into the film may be in flight on any stream
  VPT_HIP(hipMemsetAsync(ctx->film, 0, ctx->film_count * sizeof(float), ctx->stream));
  VPT_HIP(hipStreamSynchronize(ctx->stream));
  return VPT_OK;
}

int vpt_gpu_film_device_ptr(vpt_gpu_ctx* ctx, float** film_device, uint64_t* count) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (film_device) *film_device = ctx->film;
  if (count) *count = ctx->film_count;
  return VPT_OK;
}

int vpt_gpu_film_add_to_host(vpt_gpu_ctx* ctx, float* film_host) {
  if (!ctx || !film_host) return vpt::set_error(VPT_E_INVALID, "null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;
  std::vector<float> tmp(ctx->film_count);
  VPT_HIP(hipMemcpy(tmp.data(), ctx->film, ctx->film_count * sizeof(float), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < ctx->film_count; ++i) film_host[i] += tmp[i];
  return VPT_OK;
}

int vpt_gpu_counters(vpt_gpu_ctx* ctx, vpt_counters* out, int reset) {
  if (!ctx || !out) return vpt::set_error(VPT_E_INVALID, "null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;
  unsigned long long c[vpt::kCounterCount];
  VPT_HIP(hipMemcpy(c, ctx->counters, sizeof c, hipMemcpyDeviceToHost));
  uint64_t* o = reinterpret_cast<uint64_t*>(out);
  for (int i = 0; i < vpt::kCounterCount; ++i) o[i] = c[i];
  if (reset) VPT_HIP(hipMemset(ctx->counters, 0, sizeof c));
  return VPT_OK;
}

int vpt_gpu_set_tuning(vpt_gpu_ctx* ctx, int gate_min, int gate_idle, int grid_blocks, int gate_eval, int gate_walk) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  // gate_idle >= 1 is what guarantees progress: with no lane walking, every waiting block runs.
  if (gate_idle == 0) return vpt::set_error(VPT_E_INVALID, "gate_idle must be >= 1 (0 can stall a wavefront)");
  if (gate_eval > 0) ctx->scene.gate_eval = gate_eval;
  if (gate_walk >= 0) ctx->scene.gate_walk = gate_walk;
  if (gate_min > 0) ctx->scene.gate_min = gate_min;
  if (gate_idle >= 0) ctx->scene.gate_idle = gate_idle;
  if ((rc = push_scene(ctx))) return rc;
  if (grid_blocks > 0) {
    ctx->grid_blocks = grid_blocks;
    ctx->grid_user = true;
  }
  return VPT_OK;
}

int vpt_gpu_set_latency_tuning(vpt_gpu_ctx* ctx, int wave_lanes, int gate_min, int gate_idle, int gate_eval,
                               int gate_walk) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (wave_lanes > 64) return vpt::set_error(VPT_E_INVALID, "wave_lanes must be <= 64");
  if (gate_idle == 0) return vpt::set_error(VPT_E_INVALID, "gate_idle must be >= 1 (0 can stall a wavefront)");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if (wave_lanes >= 0) ctx->lat_wave_lanes = wave_lanes;
  if (gate_min > 0) ctx->lat_gate[0] = gate_min;
  if (gate_idle >= 0) ctx->lat_gate[1] = gate_idle;
  if (gate_eval > 0) ctx->lat_gate[2] = gate_eval;
  if (gate_walk >= 0) ctx->lat_gate[3] = gate_walk;
  return push_scene(ctx);
}

int vpt_gpu_set_latency_kernel(vpt_gpu_ctx* ctx, int mode, int ungated) {
  if (!ctx || mode < -1 || mode > 1 || ungated < -1 || ungated > 1)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_latency_kernel: bad argument");
  ctx->lat_mode = mode;  // read by the next render's host code only: no wait
  if (ungated >= 0) ctx->lat_ungated = ungated;
  return VPT_OK;
}

int vpt_gpu_profile(vpt_gpu_ctx* ctx, uint64_t* out, int n, int reset) {
  if (!ctx || !out) return vpt::set_error(VPT_E_INVALID, "null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;
  std::vector<unsigned long long> v(kProfWords);
  VPT_HIP(hipMemcpy(v.data(), ctx->prof, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  if (n < (int)v.size()) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_profile: output too small");
  for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
  if (reset) VPT_HIP(hipMemset(ctx->prof, 0, v.size() * sizeof(unsigned long long)));
  return VPT_OK;
}

int vpt_gpu_launch_info(const vpt_gpu_ctx* ctx, int* grid_blocks, int* block_threads) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (grid_blocks) *grid_blocks = ctx->grid_blocks;
  if (block_threads) *block_threads = vpt::kBlockThreads;
  return VPT_OK;
}

int vpt_gpu_set_compaction(vpt_gpu_ctx* ctx, int every) {
  if (!ctx || every < 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_compaction: bad argument");
  ctx->compact_every = every;  // read by the next render's host code only: no wait
  return VPT_OK;
}

int vpt_gpu_latency_kernel_info(const vpt_gpu_ctx* ctx, int* mode, int* resident_blocks_per_cu) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (mode) *mode = ctx->lat_mode;
  if (resident_blocks_per_cu) *resident_blocks_per_cu = ctx->lat_per_cu;
  return VPT_OK;
}

}  // extern "C"
