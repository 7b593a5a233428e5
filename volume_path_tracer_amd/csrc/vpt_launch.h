// vpt_launch.h — constants shared by the integrator's kernels (vpt_kernels.h) and the host code that launches
// and feeds them (vpt_gpu.hip, vpt_feed.cpp): the block size and the feed protocol's words and marks.
#pragma once

#include <cstdint>

namespace vpt {

constexpr int kBlockThreads = 256;
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

}  // namespace vpt
