// dladmm_queue.h -- the bf16 mode's whole forward as ONE persistent launch whose workgroups pull
// tile units from per-XCD work queues in dependency order (dladmm_tile_bf16_queue.hip).
#pragma once

#include "dladmm_internal.h"

namespace dladmm {

// Phases q = 0 .. nph-1: 0 the prologue (PH 2), 2k+1 G1(k) (PH 0), 2k+2 G2(k) (PH 1); a unit is
// (phase q, column tile c, row tile r).  Column tiles are dealt to 8 queues (c % 8), each ordered
// along diagonals: step t holds phase t - l of the columns of lag class l = (c / 8) % lags.
struct QueueArgs {
  const LayerArgs* ph;  // device table of the nph phases' arguments
  int nph, gx;          // phases; column tiles (256 columns each)
  int rows1, rows2;     // row tiles of a G1 / G2-shaped phase
  int lags;             // diagonal lag classes (1 = phase after phase)
  int* tickets;         // next ticket of queue x at tickets[32 x] (one 128-B line each)
  int* done;            // finished units of (q, c) at done[q * gx + c]
  int* err;             // set when a dependency wait timed out (results then invalid)
};

// words of the counter block: 8 ticket lines + nph * gx completion counts + the error word
inline int64_t queue_counter_words(int nph, int gx) { return 8 * 32 + (int64_t)nph * gx + 1; }

// dst[0 .. n) = host[0 .. n), the values travelling as kernel arguments (graph-capturable)
hipError_t write_layer_table(const LayerArgs* host, int n, LayerArgs* dst, hipStream_t s);

// grid = persistent workgroups (one per CU: 8 waves, 128 KiB of LDS ring)
hipError_t launch_tile_bf16_queue(int variant, const QueueArgs& q, int grid, hipStream_t s);

// after the queue launch: if a dependency wait timed out, poison z_last[0] and lossp[i * stride]
// for i < rows (NaN), so a failed schedule never returns plausible numbers
hipError_t launch_queue_check(const QueueArgs& q, float* z_last, float* lossp, int rows,
                              int64_t stride, hipStream_t s);

}  // namespace dladmm
