// sgd_tile.hip -- K1 tile schedule (RS_SGD_WB_TILE, the FAST default): the SGD epoch of the Funk-SVD
// model (reference core/svd.go:92-130) with the user rows held in LDS and the item rows combined
// per workgroup, gfx950.
//
// Why (measured): every schedule that writes each rating's q_i update to memory is
// bound by the memory-side atomic unit (u32 adds 1.69 TB/s on gfx950, float adds 1.3 TB/s: one
// 448-B row per rating at k = 100 is 0.45 GB per ML-1M epoch, >= 265 us).  Integer LDS atomics, on
// the other hand, run at the LDS write rate (scripts/experiments/exp_lds_atomics.hip: ds_add_u32
// 8.7 cycles per 512-B row per CU at 16 waves, the same as ds_write_b32; ds_add_f32 is 44x slower).
// So the epoch is reorganised around them:
//
//   * Users are cut into TILES (consecutive users, about nnz / #CUs ratings each, bounded by the
//     LDS).  One workgroup of NW waves owns a tile at a time: its P rows are staged into LDS as
//     int32 fixed point round(p * 2^S) and every p_u update is a ds_add_u32 of the rounded delta --
//     exact and order-free, so the NW waves share the rows without locks (Hogwild inside the CU, no
//     update lost).  Tiles hold disjoint users, so P needs no cross-CU coherence at all.
//   * The tile's ratings are grouped into RUNS, one per item (the item's ratings by the tile's
//     users).  A wave takes a run, loads q_i once (an sc1 load of the int32 row), applies the run's
//     ratings one after the other with q_i in VGPRs -- the sequential update order of svd.go:97-128
//     inside the run, including the aliasing Q1 (q_i moves with the NEW p_u) -- and adds the
//     run's total delta to memory with one integer atomic per row line.  The memory-side traffic
//     per epoch drops from one row per rating to one row per (item, tile) pair: 1.0M -> 0.44M rows
//     on the ML-1M shape with 256 tiles.
//   * Runs are dealt to the waves of a tile in a per-tile pseudo-random order (longest-first
//     balancing over waves), so a hot item's runs are spread over the epoch in time: the staleness
//     of a hot q_i (updates other workgroups hold in registers while this one reads it) stays at
//     ~ deg * run time / epoch, a few tens of ratings, like the per-rating schedules.
//
// GlobalBias (Q2) is a per-(tile, wave) local SGD copy from the epoch-start value, folded at epoch end.  The
// single-GPU epoch folds the streams' chains smoothed (round 6; sgd.hip svd_epoch_epilogue_kernel): each stream's
// chain gb <- (1 - lr) gb - lr e_j over its n ratings is the map gb0 -> a gb0 + b, a = (1 - lr)^n, so
// T = sum b / sum (1 - a) is the common level the streams pull toward, and gb' = A gb0 + (1 - A) T with
// A = (1 - lr)^nnz -- the sequential chain with its e_j at their mean.  The multi-GPU exchanges keep the mean of
// the moves (gb += sum n_w (gb_w - gb) / nnz, fixed order), as the other FAST schedules do.  A user too heavy for one tile's LDS is cut into
// pieces in different tiles, each from the same p_u, merged by count-weighted average after the
// epoch (as rs_svd_plan_set_split).
//
// Visit order: tile by tile, a tile's runs in their dealt order, a run's ratings in user order.  With
// one workgroup of one wave the kernel is the sequential SGD in that order (rs_svd_plan_tile_order
// exports it; tests/test_tile_gpu.py restates it with the ORDERED oracle).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <queue>
#include <utility>
#include <stdexcept>
#include <thread>
#include <vector>

#include "common.hpp"
#include "sgd_plan.hpp"
#include "wave.hpp"

namespace rs {


// Wave sum ending in lane 63 (GFX9 DPP row broadcasts): the in-row tree gives every lane its row's
// sum, row_bcast:15 adds row 0 / 2's sum into rows 1 / 3, row_bcast:31 adds rows 0-1 into rows 2-3.
// Six VALU ops and a v_readlane, against ten for the all-lanes form (the value is needed as a scalar).
__device__ __forceinline__ float wave_sum_l63(float x) {
    x = group_sum<16>(x);
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xA, 0xF, false));  // row_bcast:15
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

// floor(x + 0.5) as int32 in one VALU op (v_cvt_rpi_i32_f32; __float2int_rn is rndne + cvt)
__device__ __forceinline__ int32_t cvt_rpi(float x) {
    int32_t r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// Register layout of the tile kernel: lane l's register x holds logical column c = l + 64 x.  Columns
// [0, k) are the factors; the biases fold into the dot product with a constant partner column:
//   P row: [p_0 .. p_{k-1}, b_u, 1]     Q row: [q_0 .. q_{k-1}, 1, b_i]
// so p.q over all columns = p.q + b_u + b_i, and the one update formula p <- a p - c q,
// q <- a q - c p_new gives b_u <- a b_u - c and b_i <- a b_i - c (svd.go:108-112); only the two
// constant columns are held at 1 by a select.  In memory the bias sits in column k of both rows
// (the 64-B line budget of the global atomics, sgd.hip) and nothing is stored past it.
//
// Work distribution inside a tile (CH, round 4).  CH = 0: the runs are dealt to the NW waves on the host
// (streams of near-equal ratings).  CH > 0: the tile's runs form ONE queue and a wave claims CH
// consecutive runs at a time from an LDS counter.  Round 3's per-wave clocks showed that a
// wave's time does not follow its ratings or runs (R^2 = 0.04) but the memory side, so no static deal can
// balance it: the slowest of 16 waves was 8 % above the mean.  With claims a workgroup ends about one
// chunk after its mean wave.  The claim for the chunk after next is issued when a chunk starts and its
// headers / first record window are read after the chunk's first / second run, so no LDS round trip
// waits on the critical path.  With one wave the claims come in queue order: the visit order is the
// queue, as rs_svd_plan_tile_order exports it.
template <int E, int NW, int RQ, int CH, int DIAG = 0, bool DAMP = false, bool COLD = false>
__global__ __launch_bounds__(NW * 64) void svd_epoch_tile_kernel(
    const int4* __restrict__ tiles, int32_t n_tiles, const int2* __restrict__ tile_users,
    const int32_t* __restrict__ streams, const int2* __restrict__ runs, const int2* __restrict__ recs,
    float* __restrict__ P, int32_t* Q, int32_t q_bytes, const double* __restrict__ gb_in,
    double* __restrict__ gb_partial, float* __restrict__ loss_partial, float lr, float reg, float fx, float* __restrict__ dP,
    const float* __restrict__ uw, float* __restrict__ dPs, int32_t kf, int32_t ldm, int32_t ldd,
    int64_t* __restrict__ dbg, const int32_t* __restrict__ item_deg, int32_t deg_bytes, float kconc,
    double* __restrict__ gb_smooth, double l1) {
#pragma clang fp contract(fast)
    constexpr int LD = 64 * E, NT = NW * 64;  // LD: LDS row (k + 2 columns fit); ldm: the rows in HBM
    constexpr bool TIMED = (DIAG & 16) != 0;  // per-wave phase clocks into dbg (experiments)
    constexpr bool SPAN = (DIAG & 32) != 0;   // per-wave start / end clocks only (no extra waits)
    static_assert(CH == 0 || (CH > RQ && CH >= 2 && CH < 64), "a claimed chunk must outlast the ring");
    // the chunk loop steps the ring RQ runs at a time: a ring that does not divide the chunk would train
    // runs of the next chunk here (the wave that claims it trains them again) and misalign the slots
    static_assert(CH == 0 || CH % RQ == 0, "a claimed chunk must be a whole number of ring turns");
    int64_t tm_stage = 0, tm_ring = 0, tm_loop = 0, tm_tail = 0, tm_c = 0;
    auto clk = [] { return static_cast<int64_t>(__builtin_amdgcn_s_memtime()); };
    static_assert((2 * E + (DAMP ? 1 : 0)) * RQ <= 60, "ring loads and atomics must fit the 63-op vmcnt");
    typedef float f2 __attribute__((ext_vector_type(2)));
    extern __shared__ __align__(16) int32_t lds[];
    __shared__ int32_t s_claim;  // CH > 0: next unclaimed chunk of the tile's run queue
    const int tid = static_cast<int>(threadIdx.x), lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    // the items' degrees (hot-run damping): loaded with each run's q_i row, in order on the same vmcnt
    const __amdgpu_buffer_rsrc_t rdeg =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(item_deg), 0, item_deg ? deg_bytes : 0, 0x00020000);
    const double gb0 = gb_in[0];
    const float a = 1.f - lr * reg, am1 = -lr * reg, fx_inv = 1.f / fx;
    // per register: global byte offset of this lane's Q element in a row (-1: none), constant lanes
    int32_t qoff[E];
    bool qone[E], pone[E], pfac[E];
#pragma unroll
    for (int x = 0; x < E; ++x) {
        const int32_t c = lane + 64 * x;
        qoff[x] = c < kf ? 4 * c : (c == kf + 1 ? 4 * kf : -1);
        qone[x] = c == kf;      // Q's constant 1 (partner of b_u)
        pone[x] = c == kf + 1;  // P's constant 1 (partner of b_i); Q's b_i
        pfac[x] = c < kf;       // a factor column
    }
    auto qaddr = [&](int32_t row, int x) { return (row >= 0 && qoff[x] >= 0) ? row + qoff[x] : kOutOfRange; };
    double contrib = 0.0;
    double s_num = 0.0, s_den = 0.0;  // the smoothed GlobalBias fold's sums (gb_smooth != nullptr; sgd.hip epilogue)
    float se = 0.f;  // sum of c^2 = (lr diff)^2 over this wave's ratings: the epoch's training loss (the guard)
    const int64_t t_begin = SPAN ? clk() : 0;
    const int64_t rt_begin = SPAN ? static_cast<int64_t>(__builtin_amdgcn_s_memrealtime()) : 0;  // 100 MHz, chip-wide

    for (int32_t t = static_cast<int32_t>(blockIdx.x); t < n_tiles; t += static_cast<int32_t>(gridDim.x)) {
        if constexpr (TIMED) tm_c = clk();
        const int4 tm = tiles[t];  // {first user entry, entries, first run, first record}
        const int32_t nu = tm.y;
        const int32_t* sp = streams + static_cast<int64_t>(t) * (NW + 1);
        const int32_t n_runs = sp[NW];
        const int2* tr = runs + tm.z;  // n_runs + 1 entries: a sentinel holds the record count
        const int32_t n_rec = tr[n_runs].y;
        int32_t* Pl = lds;
        int2* Rl = reinterpret_cast<int2*>(Pl + nu * LD);
        int2* Ul = Rl + n_rec;
        auto load_q = [&](int32_t (&q)[E], int32_t& dg, int32_t item) {
            const int32_t row = item >= 0 ? (item & kRunItemMask) * (ldm * 4) : -1;  // SGPR arithmetic
#pragma unroll
            for (int x = 0; x < E; ++x)
                q[x] = (DIAG & 2) ? 0
                                  : static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(rq, qaddr(row, x), 0, kSgdAux));
            if constexpr (DAMP)
                dg = static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(rdeg, item >= 0 ? (item & kRunItemMask) * 4 : kOutOfRange, 0, 0));
            else
                dg = 0;
        };
        int32_t ring[RQ][E], ringd[RQ];
        auto prefill = [&](auto&& item_at) {
#pragma unroll
            for (int s = 0; s < RQ; ++s) {
                load_q(ring[s], ringd[s], item_at(s));
                // dropped atomics (out-of-range offsets): the loop is entered with the same pattern of
                // loads and atomics in flight as its back edge carries, so the compiler's vmcnt waits
                // keep the whole ring in flight instead of draining to the prologue's count
#pragma unroll
                for (int x = 0; x < E; ++x) {  // per-lane offsets and value: not folded into one lane
                    int32_t z;
                    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
                    __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(z, rq, kOutOfRange + lane * 4 + 256 * x, 0, 0);
                }
            }
        };
        // claimed runs: the wave's first chunk (chunk w) comes from the run headers in HBM, so its q_i rows
        // load while the tile is staged (one memory latency instead of two before the first run)
        int2 hn0 = make_int2(-1, 0);
        if constexpr (CH > 0) {
            hn0 = tr[min(w * CH + lane, n_runs)];
            prefill([&](int s) { return __builtin_amdgcn_readlane(hn0.x, s); });
        }
        // stage the tile: P rows as int32 fixed point in the register layout above, records, runs
        for (int32_t x = tid; x < nu * LD; x += NT) {
            const int32_t ul = x / LD, c = x - ul * LD;
            int32_t v = 0;
            if (c <= kf) v = __float2int_rn(P[static_cast<int64_t>(tile_users[tm.x + ul].x) * ldm + c] * fx);
            else if (c == kf + 1) v = static_cast<int32_t>(fx);
            Pl[x] = v;
        }
        for (int32_t x = tid; x < n_rec; x += NT) Rl[x] = recs[tm.w + x];
        for (int32_t x = tid; x <= n_runs; x += NT) Ul[x] = tr[x];
        if (CH > 0 && tid == 0) s_claim = NW;  // chunk w is wave w's without a claim
        __syncthreads();
        if constexpr (TIMED) {
            const int64_t c = clk();
            tm_stage += c - tm_c;
            tm_c = c;
        }

        // Records are read from LDS in 64-entry windows (one lane-parallel read per 64 ratings, then
        // v_readlane with an SGPR index): no LDS round trip per rating.
        int32_t rb = 0, j = 0;  // record window base, next record (tile-local)
        int2 rw0, rw1;
        auto set_window = [&](int32_t first) {
            rb = j = first;
            rw0 = Rl[min(rb + lane, n_rec - 1)];
            rw1 = Rl[min(rb + 64 + lane, n_rec - 1)];
        };
        double gb = gb0;
        const float klr = lr * fx_inv * fx_inv;  // c = lr (s 2^-2S + gb - r): p and q in 2^-S units (S: the plan's shift)
        // One run: its q_i row comes out of ring slot `slot`, which is refilled with the row of `next`;
        // records [j, e) are trained in order with q_i in registers, then the run's delta goes to memory.
        auto run = [&](int32_t (&slot)[E], int32_t& slotd, int32_t item, int32_t e, int32_t next) {
            int64_t c0 = 0;
            if constexpr (TIMED) c0 = clk();
            // Hot-run damping (round 5).  About R = deg_i x workgroups x waves / nnz runs of item i are in flight
            // at any time (the item's share of the ratings the chip's waves hold), each from a q_i read before the
            // others' deltas land.  Where their summed step would pass the gap sequential SGD closes -- R times
            // this run's own closing fraction f = 1 - prod(1 - lr (|p_u|^2 + reg)) over its ratings, beyond 1 --
            // the run's delta is scaled by 1 / (R f) (the bias column: f from 1 - lr (1 + reg) per rating).
            // Only runs with R >= 4 measure |p_u|^2 (an extra wave sum per rating); with one wave per tile, or
            // the runs of an ML-1M epoch (R <= 10, R f < 1), nothing changes.  DESIGN.md K1 round 5.
            const float R = DAMP ? static_cast<float>(__builtin_amdgcn_readfirstlane(slotd)) * kconc : 0.f;
            const bool hot = DAMP && R >= 4.f;
            const int32_t n_run = e - j;
            float hp = 0.f;  // this lane's columns of the run's sum of |p_u|^2, in 2^-2S units
            int32_t q0[E];
            float q[E];
#pragma unroll
            for (int x = 0; x < E; ++x) {
                // a real copy: the slot is then dead and its refill lands in the same registers (a
                // coalesced copy would keep both live and the compiler would rotate the ring with
                // moves at the loop back edge, waiting for every load in flight there)
                asm volatile("v_mov_b32 %0, %1" : "=v"(q0[x]) : "v"(slot[x]));
                q[x] = qone[x] ? fx : static_cast<float>(q0[x]);  // q in 2^-S units too
            }
            if constexpr (TIMED) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (timed variant only) honest split
                const int64_t c1 = clk();
                tm_ring += c1 - c0;
                c0 = c1;
            }
            load_q(slot, slotd, next);  // refill: every slot issues E + 1 loads + E atomics
            const float gbf = static_cast<float>(gb);
            float cs = 0.f;  // sum of this run's c: GlobalBias moves by -cs (folded in double)
            for (; j < e; ++j) {
                if (j - rb >= 64) {  // slide the record window (every 64 ratings)
                    rb += 64;
                    rw0 = rw1;
                    rw1 = Rl[min(rb + 64 + lane, n_rec - 1)];
                }
                const int32_t o = j - rb;
                const int32_t ul = __builtin_amdgcn_readlane(rw0.x, o);
                const float rt = __int_as_float(__builtin_amdgcn_readlane(rw0.y, o));
                int32_t* prow = Pl + ul * LD + lane;
                float pu[E];  // p in 2^-S units
#pragma unroll
                for (int x = 0; x < E; ++x)
                    pu[x] = (DIAG & 8) ? 1e5f * ul : static_cast<float>(prow[64 * x]);
                // dot over all columns (biases included), two columns per packed op
                float sd;
                {
                    f2 acc = {0.f, 0.f};
#pragma unroll
                    for (int x = 0; x + 1 < E; x += 2) {
                        const f2 pv = {pu[x], pu[x + 1]}, qv = {q[x], q[x + 1]};
                        acc = __builtin_elementwise_fma(pv, qv, acc);
                    }
                    sd = acc.x + acc.y;
                    if constexpr (E & 1) sd = __builtin_fmaf(pu[E - 1], q[E - 1], sd);
                }
                sd = wave_sum_l63(sd);
                if (hot) {  // per lane; summed over the wave once, at the run's end
#pragma unroll
                    for (int x = 0; x < E; ++x)
                        if (pfac[x]) hp = __builtin_fmaf(pu[x], pu[x], hp);
                }
                // svd.go:102-128: diff = (gb + b_u + b_i + p.q) - r, c = lr diff;
                // p <- a p - c q ; q <- a q - c p_new (Q1) ; gb <- gb - c
                const float c = __builtin_fmaf(sd, klr, lr * ((gbf - cs) - rt));
                cs += c;
                se = __builtin_fmaf(c, c, se);

                float pn[E];
#pragma unroll
                for (int x = 0; x + 1 < E + 1; x += 2) {
                    if (x + 1 < E) {  // d = (a - 1) p - c q in 2^-S units; p_new = p + d
                        const f2 pv = {pu[x], pu[x + 1]}, qv = {q[x], q[x + 1]};
                        f2 d = __builtin_elementwise_fma(qv, f2{-c, -c}, pv * f2{am1, am1});
                        if (pone[x]) d.x = 0.f;  // P's constant column stays 1 (b_i's partner)
                        if (pone[x + 1]) d.y = 0.f;
                        const f2 np = pv + d;
                        const f2 nq = __builtin_elementwise_fma(np, f2{-c, -c}, qv * f2{a, a});
                        pn[x] = d.x;
                        pn[x + 1] = d.y;
                        q[x] = nq.x;
                        q[x + 1] = nq.y;
                    } else {
                        const float d = pone[x] ? 0.f : __builtin_fmaf(q[x], -c, pu[x] * am1);
                        pn[x] = d;
                        q[x] = __builtin_fmaf(pu[x] + d, -c, q[x] * a);
                    }
                }
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    if (qone[x]) q[x] = fx;
                    const int32_t di = cvt_rpi(pn[x]);
                    if (!(DIAG & 4))
                        __hip_atomic_fetch_add(prow + 64 * x, di, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            gb -= static_cast<double>(cs);
            if constexpr (TIMED) tm_loop += clk() - c0;
            const int32_t row = item >= 0 ? (item & kRunItemMask) * (ldm * 4) : -1;
            // a cold item's run (header bit kRunCold, sgd_plan.hpp): hardly any other run of the item is in flight, so
            // the new row is written through with plain sc1 stores instead of memory-side atomics (round 6)
            const bool cold = COLD && item >= 0 && (item & kRunCold) != 0;
            bool damp = false;  // wave-uniform: the common path keeps its exact integer delta and no extra work
            float wq = 1.f, wb = 1.f;
            if (hot) {
                hp = wave_sum_l63(hp);
                const float fq = 1.f - __expf(-lr * (hp * fx_inv * fx_inv + static_cast<float>(n_run) * reg));
                const float fb = 1.f - __expf(static_cast<float>(n_run) * __logf(1.f - lr * (1.f + reg)));
                wq = fminf(1.f, 1.f / (R * fq));
                wb = fminf(1.f, 1.f / (R * fb));
                damp = wq < 1.f || wb < 1.f;
            }
            if (damp) {
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    const float wx = pone[x] ? wb : wq;
                    const int32_t dq = cvt_rpi(wx * (q[x] - static_cast<float>(q0[x])));
                    if constexpr (DIAG & 1)
                        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(dq, rq, kOutOfRange + lane * 4 + 256 * x, 0, 0);
                    else
                        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(dq, rq, qaddr(row, x), 0, 0);
                }
            } else if (cold && !(DIAG & 1)) {  // the same E vector memory ops per run as the atomics (vmcnt)
#pragma unroll
                for (int x = 0; x < E; ++x)
                    __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(cvt_rpi(q[x])), rq, qaddr(row, x), 0, kSgdAux);
            } else {
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    const int32_t dq = cvt_rpi(q[x]) - q0[x];
                    if constexpr (DIAG & 1)  // diagnostic: the atomic goes nowhere (same issue count)
                        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(dq, rq, kOutOfRange + lane * 4 + 256 * x, 0, 0);
                    else
                        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(dq, rq, qaddr(row, x), 0, 0);
                }
            }
        };

        int32_t nr = 0;  // ratings this wave trained in this tile (the GlobalBias fold's weight)
        if constexpr (CH == 0) {
            const int32_t r0 = sp[w], r1 = sp[w + 1];
            // Run headers are read from LDS in 64-entry windows like the records
            int32_t hb = r0;  // run window base: lane l of (hw0, hw1) holds run hb + l, hb + 64 + l
            int2 hw0 = Ul[min(hb + lane, n_runs)], hw1 = Ul[min(hb + 64 + lane, n_runs)];
            auto run_hdr = [&](int32_t r, bool want_begin) -> int32_t {  // item or first record of run r
                const int32_t o = r - hb;
                const int32_t v = o < 64 ? (want_begin ? hw0.y : hw0.x) : (want_begin ? hw1.y : hw1.x);
                return __builtin_amdgcn_readlane(v, o & 63);
            };
            auto item_of = [&](int32_t r) -> int32_t { return r < r1 ? run_hdr(r, false) : -1; };
            const int32_t s_end = __builtin_amdgcn_readfirstlane(Ul[r1].y);  // records [first of r0, first of r1)
            const int32_t s_begin = run_hdr(r0, true);
            set_window(s_begin);
            prefill([&](int s) { return item_of(r0 + s); });
            for (int32_t r = r0; r < r1; r += RQ) {
#pragma unroll
                for (int s = 0; s < RQ; ++s) {
                    const int32_t rr = r + s;
                    const bool live = rr < r1;  // wave-uniform
                    if (live && rr - hb >= 64) {  // slide the run window (every 64 runs)
                        hb += 64;
                        hw0 = hw1;
                        hw1 = Ul[min(hb + 64 + lane, n_runs)];
                    }
                    const int32_t item = live ? run_hdr(rr, false) : -1;
                    const int32_t e = live ? run_hdr(rr + 1, true) : j;
                    run(ring[s], ringd[s], item, e, item_of(rr + RQ));
                }
            }
            nr = s_end - s_begin;
        } else {
            // chunk c holds runs [c CH, c CH + CH) of the queue; lane l of a header window holds run c CH + l
            // (the sentinel past the last run: item -1, first record n_rec -- an empty run)
            const int32_t n_chunks = (n_runs + CH - 1) / CH;
            auto hdr = [&](int32_t c) { return Ul[min(c * CH + lane, n_runs)]; };
            auto hx = [](const int2& h, int i) { return __builtin_amdgcn_readlane(h.x, i); };
            auto hy = [](const int2& h, int i) { return __builtin_amdgcn_readlane(h.y, i); };
            int32_t cn = w, claim = 0;
            int2 hn = hn0;  // = hdr(cn), read from HBM before the staging barrier (its ring is in flight)
            int2 rwn = Rl[min(hy(hn, 0) + lane, n_rec - 1)];  // the next chunk's first record window
            while (true) {
                const int32_t cc = cn;
                const int2 hc = hn;
                if (cc >= n_chunks) break;
                rb = j = hy(hc, 0);
                rw0 = rwn;
                rw1 = Rl[min(rb + 64 + lane, n_rec - 1)];
                nr += hy(hc, CH) - j;
                if (lane == 0) claim = atomicAdd(&s_claim, 1);  // the chunk after this one
#pragma unroll
                for (int p0 = 0; p0 < CH; p0 += RQ) {
#pragma unroll
                    for (int s = 0; s < RQ; ++s) {
                        const int p = p0 + s;
                        const int32_t nxt = p + RQ < CH ? hx(hc, p + RQ) : hx(hn, p + RQ - CH);
                        run(ring[s], ringd[s], hx(hc, p), hy(hc, p + 1), nxt);
                        if (p == 0) {  // the claim has landed behind this run's LDS traffic
                            cn = __builtin_amdgcn_readfirstlane(claim);
                            hn = hdr(cn);
                        } else if (p == 1) {
                            rwn = Rl[min(hy(hn, 0) + lane, n_rec - 1)];
                        }
                    }
                }
            }
        }
        if constexpr (TIMED) tm_c = clk();
        contrib += static_cast<double>(nr) * (gb - gb0);
        if (gb_smooth) {  // this stream's chain gb0 -> gb over nr ratings: gb = a gb0 + b, a = (1 - lr)^nr
            const double an = exp(static_cast<double>(nr) * l1);
            s_num += gb - an * gb0;
            s_den += 1.0 - an;
        }
        __syncthreads();
        // write the tile's P rows back: whole users stored (or their weighted delta to dP in
        // multi-GPU delta mode), pieces of split users as count-weighted deltas
        for (int32_t x = tid; x < nu * LD; x += NT) {
            const int32_t ul = x / LD, c = x - ul * LD;
            if (c > kf) continue;  // the constant column and padding are not stored
            const int2 te = tile_users[tm.x + ul];  // {user, frac bits}
            const float frac = __int_as_float(te.y);
            const int64_t g = static_cast<int64_t>(te.x) * ldm + c;
            const float v = fx_to_f(static_cast<uint32_t>(Pl[x]), fx_inv);
            if (dP) {  // multi-GPU delta mode: dP rows of stride ldd
                const float d = uw[te.x] * frac * (v - P[g]);
                const int64_t gd = static_cast<int64_t>(te.x) * ldd + c;
                if (frac == 1.f) dP[gd] = d;
                else atomicAdd(dP + gd, d);
            } else if (frac == 1.f) {
                P[g] = v;
            } else {
                atomicAdd(dPs + g, frac * (v - P[g]));
            }
        }
        __syncthreads();  // the next tile's staging overwrites the LDS
        if constexpr (TIMED) tm_tail += clk() - tm_c;
    }
    // one partial per workgroup, its waves' sums in wave order: the epilogue then folds grid values instead of
    // grid x waves (round 6: its loads were the epilogue's time, ~7 us of an ML-1M step)
    __shared__ double s_part[3][NW];
    __shared__ float s_loss[NW];
    if (lane == 0) {
        s_part[0][w] = contrib;
        s_part[1][w] = s_num;
        s_part[2][w] = s_den;
        s_loss[w] = se;
    }
    __syncthreads();
    if (tid == 0) {
        double c = 0.0, sn = 0.0, sd = 0.0;
        float sl = 0.f;
        for (int x = 0; x < NW; ++x) {
            c += s_part[0][x];
            sn += s_part[1][x];
            sd += s_part[2][x];
            sl += s_loss[x];
        }
        gb_partial[blockIdx.x] = c;
        if (gb_smooth) {
            gb_smooth[2 * static_cast<int64_t>(blockIdx.x)] = sn;
            gb_smooth[2 * static_cast<int64_t>(blockIdx.x) + 1] = sd;
        }
        if (loss_partial) loss_partial[blockIdx.x] = sl;
    }
    if constexpr (SPAN) {
        const int64_t t_end = clk();
        if (lane == 0) {
            int64_t* d = dbg + (static_cast<int64_t>(blockIdx.x) * NW + w) * 4;
            d[0] = t_begin;
            d[1] = t_end;
            const int64_t rt_end = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
            const int64_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // XCC_ID (XCD)
            d[2] = rt_begin;
            d[3] = (rt_end - rt_begin) | (xcc << 48);
        }
    }
    if constexpr (TIMED) {
        if (lane == 0) {
            int64_t* d = dbg + (static_cast<int64_t>(blockIdx.x) * NW + w) * 4;
            d[0] = tm_stage;
            d[1] = tm_ring;
            d[2] = tm_loop;
            d[3] = tm_tail;
        }
    }
}

namespace {

uint32_t mix32(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return static_cast<uint32_t>((x ^ (x >> 31)) >> 16);
}

struct TileHost {
    std::vector<int4> tiles;
    std::vector<int2> users;      // {user, frac bits}
    std::vector<int32_t> streams; // per tile NW + 1
    std::vector<int2> runs, recs;
    std::vector<int64_t> pos;     // CSR position of every record (want_pos only)
    std::vector<int32_t> split;   // users cut into pieces
    size_t lds = 0;
};

// Tiles from the host user-CSR.  Entries (user pieces) are consecutive users; a tile closes when the
// next entry would pass the rating target or the LDS bound (runs <= records).  A user whose ratings
// do not fit one tile's LDS is cut into near-equal pieces (count-weighted merge after the epoch).
void build_tile_host(const rs_svd_plan* pl, int32_t u_begin, int32_t u_end, int32_t nw, int64_t target,
                     int32_t run_cap, bool want_pos, TileHost& th) {
    const bool claim = pl->tile_claim > 0;  // one run queue per tile, claimed by the waves
    const std::vector<int64_t>& rp = pl->h_rowptr;
    const int32_t ld = tile_lds_row(pl);
    // one entry alone must fit: ld*4 + d*16 + 8 <= budget
    const int64_t rec_cap = static_cast<int64_t>((kTileLdsBudget - 16 - static_cast<size_t>(ld) * 4) / 16);
    if (rec_cap < 64) throw std::invalid_argument("n_factors too large for the tile schedule's LDS");
    struct Ent { int32_t u; int64_t b, e; float frac; };
    std::vector<Ent> ents;
    for (int32_t u = u_begin; u < u_end; ++u) {
        const int64_t d = rp[u + 1] - rp[u];
        if (d == 0) continue;
        const int64_t cap = std::min<int64_t>(rec_cap, std::max<int64_t>(target, 1));
        const int64_t pieces = d > rec_cap ? (d + cap - 1) / cap : 1;
        if (pieces > 1) th.split.push_back(u);
        for (int64_t x = 0; x < pieces; ++x) {
            const int64_t b = rp[u] + d * x / pieces, e = rp[u] + d * (x + 1) / pieces;
            ents.push_back({u, b, e, pieces > 1 ? static_cast<float>(static_cast<double>(e - b) / d) : 1.f});
        }
    }
    // Tiles by LPT over the entries (heaviest first, each to the least-loaded tile its LDS still takes):
    // near-equal ratings per tile -- the epoch is its slowest workgroup, and a workgroup's time tracks
    // its tile's ratings (measured: correlation 0.90 on the ML-1M shape).  The tile count is the
    // larger of nnz / target and what the LDS needs; entries of a tile keep user order.
    static const bool ttrace = std::getenv("RSGPU_TILE_TRACE") != nullptr;
    auto tprev = std::chrono::steady_clock::now();
    auto tmark = [&](const char* what) {
        if (!ttrace) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "tile-build %-8s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t1 - tprev).count());
        tprev = t1;
    };
    std::vector<size_t> tb{0};
    {
        int64_t total = 0;
        double bytes = 0;
        for (const Ent& x : ents) {
            total += x.e - x.b;
            bytes += static_cast<double>(ld) * 4 + 16.0 * static_cast<double>(x.e - x.b);
        }
        const int64_t n_target = (total + target - 1) / std::max<int64_t>(target, 1);
        const int64_t n_lds = static_cast<int64_t>(std::ceil(bytes / (0.85 * static_cast<double>(kTileLdsBudget))));
        const int64_t n0 = std::max<int64_t>({1, n_target, n_lds});
        if (pl->tile_rule != RS_TILE_RULE_LPT) {
            // fill rule (the device build, sched_dev.hip, restates it): entries by ratings, descending (ties by
            // user id) over T = min(n0, entries) tiles.  The first kFillSnakeRounds * T are dealt boustrophedon
            // (position p, round r = p / T: tile r even ? p % T : T - 1 - p % T); then each tile's deficit
            // against the mean load, max(0, ceil(sum / T) - load), is laid end to end in deficit order
            // (descending, ties by tile), and the remaining entries, heaviest first, are laid on that line by
            // their prefix sums: each goes to the tile whose stretch holds its midpoint.  A tile's entries in
            // user order.  (ML-1M shape, 256 tiles: max/mean tile load 1.05, against 1.36 for the deal alone
            // and 1.005 for LPT.)
            if (!th.split.empty()) throw std::invalid_argument("fill tile rule: a user above the LDS bound");
            const size_t ne = ents.size(), ntl = std::min(static_cast<size_t>(n0), ne);
            const size_t ns = std::min(ne, static_cast<size_t>(kFillSnakeRounds) * ntl);
            std::vector<size_t> order(ne);
            std::iota(order.begin(), order.end(), size_t{0});
            std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
                return ents[a].e - ents[a].b > ents[b].e - ents[b].b;
            });
            // loads in LDS bytes (4 ld per user + 16 per rating: records and run headers), so that a tile of many
            // light users stays inside the LDS; at ML-1M's 512-B rows a user weighs as much as 32 ratings
            auto wgt = [&](const Ent& x) -> int64_t { return int64_t{4} * ld + 16 * (x.e - x.b); };
            std::vector<std::vector<size_t>> bins(ntl);
            std::vector<int64_t> load(ntl, 0);
            int64_t wsum = 0;
            for (size_t p = 0; p < ne; ++p) wsum += wgt(ents[p]);
            for (size_t p = 0; p < ns; ++p) {
                const size_t r = p / ntl, i = p % ntl, t = (r & 1) ? ntl - 1 - i : i;
                bins[t].push_back(order[p]);
                load[t] += wgt(ents[order[p]]);
            }
            const int64_t mean = ntl ? (wsum + static_cast<int64_t>(ntl) - 1) / static_cast<int64_t>(ntl) : 0;
            std::vector<int64_t> def(ntl);
            for (size_t t = 0; t < ntl; ++t) def[t] = std::max<int64_t>(0, mean - load[t]);
            std::vector<size_t> lt(ntl);  // the line: tiles by deficit, descending, ties by tile
            std::iota(lt.begin(), lt.end(), size_t{0});
            std::stable_sort(lt.begin(), lt.end(), [&](size_t a, size_t b) { return def[a] > def[b]; });
            std::vector<int64_t> line(ntl + 1, 0);  // exclusive prefix of the deficits in line order
            for (size_t j = 0; j < ntl; ++j) line[j + 1] = line[j] + def[lt[j]];
            int64_t rsum = 0;
            for (size_t p = ns; p < ne; ++p) {
                const int64_t d = wgt(ents[order[p]]), m2 = 2 * rsum + d;
                // first j with 2 line[j + 1] > m2
                const size_t j = static_cast<size_t>(std::upper_bound(line.begin() + 1, line.end(), m2,
                                                                      [](int64_t v, int64_t e) { return v < 2 * e; }) -
                                                     (line.begin() + 1));
                bins[lt[std::min(j, ntl - 1)]].push_back(order[p]);
                rsum += d;
            }
            std::vector<Ent> sorted;
            sorted.reserve(ne);
            for (std::vector<size_t>& bn : bins) {
                std::sort(bn.begin(), bn.end());
                for (size_t x : bn) sorted.push_back(ents[x]);
                tb.push_back(sorted.size());
            }
            ents.swap(sorted);
        } else if (n_lds > 64 && n_lds >= 4 * n_target) {
            // LDS-bound (many tiles per workgroup, e.g. a ROTATE_Q stratum of 10M users' ratings): the launch
            // balances itself over the tiles, so fill tiles in user order to the LDS instead of LPT (which took
            // ~1 s per configs[4] stratum for nothing)
            int64_t users = 0, recs = 0;
            for (size_t x = 0; x < ents.size(); ++x) {
                const int64_t d = ents[x].e - ents[x].b;
                if (users > 0 && tile_bytes(users + 1, recs + d, recs + d, ld) > kTileLdsBudget) {
                    tb.push_back(x);
                    users = recs = 0;
                }
                ++users;
                recs += d;
            }
            if (!ents.empty()) tb.push_back(ents.size());
        } else {
        std::vector<size_t> order(ents.size());
        std::iota(order.begin(), order.end(), size_t{0});
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
            return ents[a].e - ents[a].b > ents[b].e - ents[b].b;
        });
        struct Bin { int64_t recs = 0, users = 0; std::vector<size_t> ents; };
        std::vector<Bin> bins(static_cast<size_t>(n0));
        using HE = std::pair<int64_t, size_t>;  // (ratings, bin), least first
        std::priority_queue<HE, std::vector<HE>, std::greater<HE>> heap;
        for (size_t b = 0; b < bins.size(); ++b) heap.push({0, b});
        std::vector<HE> aside;
        for (size_t x : order) {
            const int64_t d = ents[x].e - ents[x].b;
            size_t pick = SIZE_MAX;
            while (!heap.empty() && aside.size() < 8) {
                const HE h = heap.top();
                heap.pop();
                const Bin& bn = bins[h.second];
                if (tile_bytes(bn.users + 1, bn.recs + d, bn.recs + d, ld) <= kTileLdsBudget) {
                    pick = h.second;
                    break;
                }
                aside.push_back(h);
            }
            for (const HE& h : aside) heap.push(h);
            aside.clear();
            if (pick == SIZE_MAX) {  // no tile with room: a new one
                pick = bins.size();
                bins.emplace_back();
            }
            Bin& bn = bins[pick];
            bn.recs += d;
            bn.users += 1;
            bn.ents.push_back(x);
            heap.push({bn.recs, pick});
        }
        tmark("lpt");
        // Refinement by cost: a workgroup's time is ~ ratings + kRunCost * runs (one run per distinct item
        // of the tile; measured on the ML-1M shape: ~120 cycles per run against ~34 per rating, so
        // tiles of many light users -- more shared items -- are cheaper than tiles of one heavy user).
        // Move users from the costliest tile to the cheapest while that lowers the maximum.
        const size_t nb = bins.size();
        // (round 4 A/B on the bench shape: 176 us per epoch with it, 186 us without; profiles/r04_refine.txt)
        if (nb > 1 && nb <= 8192 && static_cast<double>(nb) * std::max(1, pl->n_items) <= 6.4e7) {
            // (round 4 sweep with claims: run cost 1 / 2 / 3 / 4 / 6 -> 181 / 180 / 177 / 176 / 177 us; 16 nb moves
            // instead of 4 nb: no change -- the moves have converged; profiles/r04_refine.txt)
            constexpr int64_t kRunCost = 3;
            constexpr size_t kIt = 4;
            std::vector<int32_t> cnt(nb * static_cast<size_t>(std::max(1, pl->n_items)), 0);
            std::vector<int64_t> runs(nb, 0), cost(nb, 0);
            auto row = [&](size_t b) { return cnt.data() + b * static_cast<size_t>(pl->n_items); };
            const std::vector<int32_t>& cols0 = pl->h_cols;
            const int32_t nth = static_cast<int32_t>(std::min<size_t>(static_cast<size_t>(clamp_threads(0)), nb / 8 + 1));
            parallel_run(nth, [&](int32_t th) {  // per-tile item counts (pooled threads)
                for (size_t b = static_cast<size_t>(th); b < nb; b += static_cast<size_t>(nth)) {
                    int32_t* c = row(b);
                    for (size_t x : bins[b].ents)
                        for (int64_t q = ents[x].b; q < ents[x].e; ++q) runs[b] += c[cols0[q]]++ == 0;
                    cost[b] = bins[b].recs + kRunCost * runs[b];
                }
            });
            for (size_t it = 0; it < kIt * nb; ++it) {
                const size_t hi = static_cast<size_t>(std::max_element(cost.begin(), cost.end()) - cost.begin());
                const size_t lo = static_cast<size_t>(std::min_element(cost.begin(), cost.end()) - cost.begin());
                if (hi == lo || bins[hi].ents.size() < 2) break;
                int64_t best = cost[hi];
                size_t best_k = SIZE_MAX;
                int64_t bh = 0, bl = 0;
                for (size_t kk = 0; kk < bins[hi].ents.size(); ++kk) {
                    const Ent& en = ents[bins[hi].ents[kk]];
                    const int64_t d = en.e - en.b;
                    if (cost[lo] + d >= best) continue;  // cl >= cost[lo] + d: cannot win (exact pruning)
                    if (tile_bytes(bins[lo].users + 1, bins[lo].recs + d, bins[lo].recs + d, ld) > kTileLdsBudget) continue;
                    int64_t lost = 0, gained = 0;
                    for (int64_t q = en.b; q < en.e; ++q) {
                        lost += row(hi)[cols0[q]] == 1;
                        gained += row(lo)[cols0[q]] == 0;
                    }
                    const int64_t ch = cost[hi] - d - kRunCost * lost, cl = cost[lo] + d + kRunCost * gained;
                    if (std::max(ch, cl) < best) {
                        best = std::max(ch, cl);
                        best_k = kk;
                        bh = ch;
                        bl = cl;
                    }
                }
                if (best_k == SIZE_MAX) break;
                const size_t x = bins[hi].ents[best_k];
                for (int64_t q = ents[x].b; q < ents[x].e; ++q) {
                    row(hi)[cols0[q]]--;
                    row(lo)[cols0[q]]++;
                }
                const int64_t d = ents[x].e - ents[x].b;
                bins[hi].ents.erase(bins[hi].ents.begin() + static_cast<std::ptrdiff_t>(best_k));
                bins[hi].recs -= d;
                bins[hi].users -= 1;
                bins[lo].ents.push_back(x);
                bins[lo].recs += d;
                bins[lo].users += 1;
                cost[hi] = bh;
                cost[lo] = bl;
            }
        }
        std::vector<Ent> sorted;
        sorted.reserve(ents.size());
        for (Bin& bn : bins) {
            if (bn.ents.empty()) continue;
            std::sort(bn.ents.begin(), bn.ents.end());
            for (size_t x : bn.ents) sorted.push_back(ents[x]);
            tb.push_back(sorted.size());
        }
        ents.swap(sorted);
        }
    }
    tmark("refine");
    const size_t nt = tb.size() - 1;
    // per tile: runs grouped by item in a per-tile pseudo-random item order, dealt to nw streams.
    // Two parallel passes over the tiles: (1) group each tile's records by item without a comparison
    // sort over records (distinct items through a per-thread item -> slot map, the distinct items put
    // in key order by an LSD radix sort of their 32-bit keys, records scattered in entry = user order),
    // cut and deal the runs; (2) write the records straight into the schedule's arrays at the tiles'
    // offsets.  One-shot Fit pays this on every call.
    struct Local {
        std::vector<int32_t> st;    // nw + 1 run offsets
        std::vector<int2> runs;     // {item, first record (tile-local)} + sentinel
        std::vector<int32_t> vul;   // grouped records: tile-local user entry
        std::vector<int64_t> vp;    //                  CSR position
        std::vector<int32_t> rb;    // per run (stream order): first grouped record
    };
    std::vector<Local> loc(nt);
    const std::vector<int32_t>& cols = pl->h_cols;
    const std::vector<float>& vals = pl->h_vals;
    const size_t cap = (run_cap > 0 && nw > 1) ? static_cast<size_t>(run_cap) : 0;
    auto group_one = [&](size_t t, std::vector<int32_t>& slot) {
        Local& L = loc[t];
        std::vector<int32_t> ditem, dcnt;
        for (size_t x = tb[t]; x < tb[t + 1]; ++x)
            for (int64_t p = ents[x].b; p < ents[x].e; ++p) {
                const int32_t it = cols[p];
                if (slot[it] < 0) {
                    slot[it] = static_cast<int32_t>(ditem.size());
                    ditem.push_back(it);
                    dcnt.push_back(0);
                }
                dcnt[slot[it]]++;
            }
        const size_t nd = ditem.size();
        std::vector<uint32_t> key(nd), ord(nd), tmp(nd);
        for (size_t d = 0; d < nd; ++d) {
            key[d] = run_key(ditem[d], static_cast<int32_t>(t));
            ord[d] = static_cast<uint32_t>(d);
        }
        for (int sh = 0; sh < 32; sh += 8) {  // LSD radix by key (ties: first appearance)
            uint32_t cnt[257] = {0};
            for (size_t d = 0; d < nd; ++d) cnt[((key[ord[d]] >> sh) & 255u) + 1]++;
            for (int b2 = 0; b2 < 256; ++b2) cnt[b2 + 1] += cnt[b2];
            for (size_t d = 0; d < nd; ++d) tmp[cnt[(key[ord[d]] >> sh) & 255u]++] = ord[d];
            ord.swap(tmp);
        }
        std::vector<int32_t> off(nd);  // grouped offset of each slot
        {
            int32_t acc = 0;
            for (size_t d = 0; d < nd; ++d) {
                off[ord[d]] = acc;
                acc += dcnt[ord[d]];
            }
        }
        size_t nrec = 0;
        for (int32_t c : dcnt) nrec += static_cast<size_t>(c);
        L.vul.resize(nrec);
        L.vp.resize(nrec);
        {
            std::vector<int32_t> fill(off);
            for (size_t x = tb[t]; x < tb[t + 1]; ++x)
                for (int64_t p = ents[x].b; p < ents[x].e; ++p) {
                    const int32_t o = fill[slot[cols[p]]]++;
                    L.vul[o] = static_cast<int32_t>(x - tb[t]);
                    L.vp[o] = p;
                }
        }
        for (int32_t it : ditem) slot[it] = -1;
        // runs in key order; with run_cap (and more than one wave) an item's records are cut into
        // pieces that go to different waves (two pieces in one wave's ring reach would read q_i
        // before the earlier piece's atomic landed).
        if (claim) {
            // Claimed runs: one queue in the per-tile pseudo-random key order, an item's pieces next to each
            // other (consecutive claims: the waves take them at about the same time, as the host deal's
            // streams did).  Measured on a hot-headed set (942k ratings, hottest item 1.95 %, k = 100,
            // scripts/experiments/exp_stability.py): pieces spread evenly over the queue instead -- each
            // tile then holds one of the item's runs in flight most of the time -- diverged at epoch 3-4 with
            // chunks of 4 and of 8; adjacent pieces train as the host deal does (10-epoch held-out 0.683 /
            // 0.683 against 0.686 for the reference order), at the same ML-1M epoch time.  The key order itself
            // matters: single-rating runs last, longest runs first or shortest first gave 197 / 252 / 257 us
            // per ML-1M epoch against 177 us (profiles/r04_refine.txt).
            struct QE { uint64_t at; int32_t sl, pc, pieces; };
            std::vector<QE> qv;
            qv.reserve(nd);
            for (size_t d = 0; d < nd; ++d) {
                const int32_t sl = static_cast<int32_t>(ord[d]);
                const size_t c = static_cast<size_t>(dcnt[sl]);
                const int32_t pieces = static_cast<int32_t>(cap ? std::min<size_t>((c + cap - 1) / cap, static_cast<size_t>(nw)) : 1);
                for (int32_t pc = 0; pc < pieces; ++pc) qv.push_back({key[sl], sl, pc, pieces});
            }
            std::stable_sort(qv.begin(), qv.end(), [](const QE& x, const QE& y) { return x.at < y.at; });
            int32_t rec = 0;
            for (const QE& e : qv) {
                const int64_t c = dcnt[e.sl];
                L.runs.push_back(make_int2(ditem[e.sl], rec));
                L.rb.push_back(off[e.sl] + static_cast<int32_t>(c * e.pc / e.pieces));
                rec += static_cast<int32_t>(c * (e.pc + 1) / e.pieces - c * e.pc / e.pieces);
            }
            L.st.assign(nw + 1, static_cast<int32_t>(L.runs.size()));
            L.st[0] = 0;
            L.runs.push_back(make_int2(-1, rec));  // sentinel
            return;
        }
        // Static deal: to the least-loaded stream (cost ~ ratings + a run start); the pieces of one item
        // take distinct streams.
        std::vector<int64_t> load(nw, 0);
        std::vector<std::vector<std::pair<int32_t, int32_t>>> sr(nw);  // per stream: (slot, piece)
        std::vector<uint8_t> used(nw, 0);
        for (size_t d = 0; d < nd; ++d) {
            const int32_t sl = static_cast<int32_t>(ord[d]);
            const size_t c = static_cast<size_t>(dcnt[sl]);
            const int32_t pieces = static_cast<int32_t>(cap ? std::min<size_t>((c + cap - 1) / cap, static_cast<size_t>(nw)) : 1);
            std::fill(used.begin(), used.end(), 0);
            for (int32_t pc = 0; pc < pieces; ++pc) {
                int best = -1;
                for (int s2 = 0; s2 < nw; ++s2)
                    if (!used[s2] && (best < 0 || load[s2] < load[best])) best = s2;
                used[best] = 1;
                load[best] += static_cast<int64_t>(c * (pc + 1) / pieces - c * pc / pieces) + 2;
                sr[best].push_back({sl, pc | (pieces << 16)});
            }
        }
        L.st.assign(nw + 1, 0);
        int32_t rec = 0;
        for (int s2 = 0; s2 < nw; ++s2) {
            L.st[s2] = static_cast<int32_t>(L.runs.size());
            for (const auto& e : sr[s2]) {
                const int32_t sl = e.first, pc = e.second & 0xffff, pieces = e.second >> 16;
                const int64_t c = dcnt[sl];
                const int32_t b = off[sl] + static_cast<int32_t>(c * pc / pieces);
                const int32_t n = static_cast<int32_t>(c * (pc + 1) / pieces - c * pc / pieces);
                L.runs.push_back(make_int2(ditem[sl], rec));
                L.rb.push_back(b);
                rec += n;
            }
        }
        L.st[nw] = static_cast<int32_t>(L.runs.size());
        L.runs.push_back(make_int2(-1, rec));  // sentinel
    };
    auto parallel_tiles = [&](auto&& fn, bool with_slot) {
        constexpr size_t kBuildThreads = 16;
        const int nth = static_cast<int>(std::min<size_t>(kBuildThreads, std::max<size_t>(1, nt / 8)));
        parallel_run(nth, [&](int32_t c) {  // (pooled threads, ingest.cpp)
            std::vector<int32_t> slot(with_slot ? static_cast<size_t>(std::max(1, pl->n_items)) : 0, -1);
            for (size_t t = static_cast<size_t>(c); t < nt; t += static_cast<size_t>(nth)) fn(t, slot);
        });
    };
    parallel_tiles(group_one, true);
    tmark("group");
    // offsets, then the records written in place
    th.tiles.resize(nt);
    std::vector<int64_t> rec_at(nt + 1, 0), run_at(nt + 1, 0);
    for (size_t t = 0; t < nt; ++t) {
        rec_at[t + 1] = rec_at[t] + static_cast<int64_t>(loc[t].vp.size());
        run_at[t + 1] = run_at[t] + static_cast<int64_t>(loc[t].runs.size());
    }
    if (run_at[nt] >= (int64_t{1} << 31) || rec_at[nt] >= (int64_t{1} << 31))
        throw std::invalid_argument("tile schedule: more than 2^31 runs or ratings");
    th.recs.resize(static_cast<size_t>(rec_at[nt]));
    th.runs.resize(static_cast<size_t>(run_at[nt]));
    th.streams.resize(nt * (nw + 1));
    if (want_pos) th.pos.resize(static_cast<size_t>(rec_at[nt]));
    parallel_tiles([&](size_t t, std::vector<int32_t>&) {
        Local& L = loc[t];
        int2* out = th.recs.data() + rec_at[t];
        int64_t* po = want_pos ? th.pos.data() + rec_at[t] : nullptr;
        const size_t nr = L.runs.size() - 1;
        size_t at = 0;
        for (size_t r = 0; r < nr; ++r) {
            const int32_t n = L.runs[r + 1].y - L.runs[r].y;
            for (int32_t x = 0; x < n; ++x, ++at) {
                const size_t g = static_cast<size_t>(L.rb[r] + x);
                int32_t bits;
                std::memcpy(&bits, &vals[L.vp[g]], 4);
                *out++ = make_int2(L.vul[g], bits);
                if (po) *po++ = L.vp[g];
            }
        }
        std::copy(L.runs.begin(), L.runs.end(), th.runs.begin() + run_at[t]);
        std::copy(L.st.begin(), L.st.end(), th.streams.begin() + static_cast<std::ptrdiff_t>(t * (nw + 1)));
        th.tiles[t] = make_int4(static_cast<int32_t>(tb[t]), static_cast<int32_t>(tb[t + 1] - tb[t]),
                                static_cast<int32_t>(run_at[t]), static_cast<int32_t>(rec_at[t]));
        loc[t] = Local();
    }, false);
    for (size_t t = 0; t < nt; ++t)
        th.lds = std::max(th.lds, tile_bytes(static_cast<int64_t>(tb[t + 1] - tb[t]), rec_at[t + 1] - rec_at[t],
                                             run_at[t + 1] - run_at[t] - 1, ld));
    th.users.resize(ents.size());
    for (size_t x = 0; x < ents.size(); ++x) {
        int32_t bits;
        std::memcpy(&bits, &ents[x].frac, 4);
        th.users[x] = make_int2(ents[x].u, bits);
    }
    tmark("emit");
    if (th.lds > kTileLdsBudget) throw std::logic_error("tile schedule exceeds the LDS");
}

// Run cap when the caller leaves it to the library (0): hot items' runs are cut so that the updates
// of one item held in registers by concurrent runs stay near kStaleTarget.  Model (measured on the
// ML-1M shape): an item of degree d cut into runs of c ratings is held by
// d * grid * waves / nnz runs at a time, each c/2 updates ahead of memory on average, so about
// S = d * grid * waves * c / (2 nnz); uncut runs (c = d / grid) give S = waves * d^2 / (2 nnz) -- 290 for
// ML-1M's hottest item at 16 waves, where 20-epoch training diverged; 8-rating pieces give ~100.
// The cap is at least dmax * 256 / nnz: every piece of a run ends in one atomic row on the item's
// single q_i row, and those atomics serialise at the memory side, so the hottest row gets at most
// about nnz / 256 of them per epoch -- the ratings one CU trains.  On configs[4]'s shard (k = 256,
// hottest item 3.4M of 126M ratings) the staleness model alone gives 2 and the hottest row's 1.7M
// atomic rows bound the epoch at 143 ms; caps 4 / 6 / 8 / 10 / 12 give 92 / 80 / 76 / 74 / 75 ms at the
// same held-out RMSE after five epochs (0.8815-0.8818; profiles/r03_experiments/cfg4_ring.log), and 7
// is what this rule picks.  On ML-1M (dmax 3428) it is 1 and changes nothing.
// The floor applies where the serialised atomics of the hottest row would outlast the rest of the epoch
// (round 4; it replaces round 3's 2^25-rating threshold): at the model's cap c the row takes d / c run-end
// atomics of L line requests each, ~4.9 ns per line (the 1.7M k = 256 rows of 17 lines in 143 ms above),
// while the epoch's other work is ~0.176 ns per rating per 7 lines (the ML-1M k = 100 epoch, 176 us per
// 1M ratings) plus ~20 us that no launch goes below.  The floor is taken when those atomics would take twice
// the rest of the epoch: configs[4]'s shard (1.7M x 17 lines = 142 ms against 2 x 54 ms): floor 7; the
// 1.13M-rating k = 64 sets (hottest item 1.4-1.6 %, model cap 3: 0.13 ms against 2 x 0.16 ms): no floor --
// caps 4-5 diverge there (round 3, profiles/r03_experiments/synth_cap.log; round 4, a first form of this
// criterion without the factor 2 took the floor on such a set and diverged on every grid) --; an ML-1M
// stratum of an 8-shard ROTATE_Q fit (14k ratings, the hottest item 428 of them: 7 us against 2 x 22 us):
// no floor -- cap 8 diverged there --; ML-1M: no floor.  What the model does not foresee, the divergence
// guard (plan_epochs, sgd.hip) catches: an epoch whose training loss rises, or a call that leaves the
// fixed-point range, is redone on half the workgroups with half the run cap.
// Round 6: the cap is at least kRunCapFloor.  1m_k100_r32 (tests/stability_sets.py: 942k ratings, hottest item
// 1.12 %, k = 100) takes the whole grid (its tiles need the LDS of 256 workgroups), where the model gives 4: the
// guard redid a call in 5 of 6 runs (training MSE up 12-30 % in one epoch, NaN with the guard off), at caps 3 / 4
// too, never on 176 / 192 workgroups (model 6 / 5).  Caps 8 and 12 took every 1M-rating stability set to 0 redos in
// every run, 10-14 % faster per epoch (fewer run-end row atomics); 8 keeps the 10-epoch held-out RMSE within
// 0.001 of the automatic cap's where 12 loses 0.005 on 1m_k100_hot (profiles/r06/stability_cap_floor.log).
constexpr double kStaleTarget = 100.0;
constexpr int64_t kRunCapFloor = 8;
constexpr double kAtomicLineNs = 4.9, kRatingLineNs = 0.176 / 7.0, kLaunchFloorNs = 20000.0;
int32_t auto_run_cap(const rs_svd_plan* pl, int32_t grid, int32_t waves) {
    if (waves <= 1 || pl->nnz == 0) return 0;
    std::vector<int64_t> deg(std::max(1, pl->n_items), 0);
    for (int32_t c : pl->h_cols) deg[c]++;
    return run_cap_rule(pl->nnz, *std::max_element(deg.begin(), deg.end()), grid, waves, pl->k);
}

}  // namespace

int32_t run_cap_rule(int64_t nnz, int64_t dmax, int32_t grid, int32_t waves, int32_t k) {
    if (waves <= 1 || nnz == 0) return 0;
    const double c = 2.0 * kStaleTarget * static_cast<double>(nnz) / (static_cast<double>(dmax) * grid * waves);
    const int64_t c_model = std::max<int64_t>(2, static_cast<int64_t>(c));
    const double lines = std::ceil((k + 1) / 16.0);  // 64-B line requests of a row (factors + bias)
    const double t_hot = static_cast<double>(dmax) / static_cast<double>(c_model) * lines * kAtomicLineNs;
    const double t_rest = static_cast<double>(nnz) * lines * kRatingLineNs + kLaunchFloorNs;
    const bool row_bound = t_hot > 2.0 * t_rest;
    const int64_t c_hot = row_bound ? (dmax * 256 + nnz - 1) / nnz : 0;
    return c >= 1e6 ? 0 : static_cast<int32_t>(std::max<int64_t>({kRunCapFloor, static_cast<int64_t>(c), c_hot}));
}

int32_t device_cus(const rs_ctx* ctx) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
        cus = 256;
    return cus;
}

// Workgroups of the tile launch when the caller leaves them to the library (tile_wg = 0).  The epoch is bound by
// the memory-side atomic unit -- one row atomic per (item, tile) run, DESIGN.md K1 round 5 -- and fewer tiles mean
// fewer runs, so a schedule whose tiles are set by the ratings target (they fit the LDS at nnz / grid ratings
// each) runs on 11/16 of the CUs: ML-1M shape, k = 100 (profiles/r05/k1_workgroups_sweep2.log): 256 / 192 / 176
// / 160 / 144 workgroups -> 176.5 / 154.0 / 146.8 / 147.1 / 158.5 us per epoch, held-out RMSE 0.6683-0.6686
// throughout; 128 and fewer run two tiles per workgroup (the LDS) and take 292-298 us.  A schedule whose tiles
// the LDS sets (configs[4]: 10M users) keeps every CU: its run count does not depend on the grid.  The host and
// the device builds use this same function of (n_users, nnz, k).
int32_t tile_grid0(const rs_svd_plan* pl) {
    if (pl->tile_wg > 0) return pl->tile_wg;
    const int32_t cus = device_cus(pl->ctx);
    const int32_t g = std::max(1, cus * 11 / 16);
    const double bytes = static_cast<double>(pl->n_users) * tile_lds_row(pl) * 4.0 + 16.0 * static_cast<double>(pl->nnz);
    return bytes / (0.85 * static_cast<double>(kTileLdsBudget)) <= static_cast<double>(g) ? g : cus;
}

namespace {

// Ratings per tile: nnz / workgroups, but at least the heaviest user's ratings (cutting users into
// pieces costs accuracy -- their rows are averaged after the epoch -- so small sets get fewer tiles).
int64_t tile_target_of(const rs_svd_plan* pl, int32_t grid, int32_t u_begin, int32_t u_end) {
    if (pl->tile_target > 0) return pl->tile_target;
    int64_t dmax = 0;
    for (int32_t u = u_begin; u < u_end; ++u) dmax = std::max(dmax, pl->h_rowptr[u + 1] - pl->h_rowptr[u]);
    const int64_t n = pl->h_rowptr[u_end] - pl->h_rowptr[u_begin];
    return std::max<int64_t>({64, dmax, (n + grid - 1) / std::max(1, grid)});
}

}  // namespace

// b-th bound = the first user whose ratings start at or past b/nb of all ratings (cum: n_users + 1
// cumulative counts); the same rule on every shard's global counts gives common bounds
std::vector<int32_t> user_block_bounds(const int64_t* cum, int32_t n_users, int32_t nb) {
    std::vector<int32_t> out(1, 0);
    for (int32_t b = 1; b < nb; ++b) {
        const int64_t want = cum[n_users] * b / nb;
        const int32_t u = static_cast<int32_t>(std::lower_bound(cum, cum + n_users + 1, want) - cum);
        out.push_back(std::max(out.back(), std::min(u, n_users)));
    }
    out.push_back(n_users);
    return out;
}

namespace {

// User blocks: tile_ublocks consecutive user ranges of near-equal ratings, tiled one after the other
// (block b's tiles are [block_tile[b], block_tile[b+1])).  One block: the plain tile schedule.
void append_tiles(TileHost& th, TileHost&& part, bool first) {
    if (first) {
        th = std::move(part);
        return;
    }
    const int32_t e0 = static_cast<int32_t>(th.users.size());
    const int64_t r0 = static_cast<int64_t>(th.runs.size()), c0 = static_cast<int64_t>(th.recs.size());
    if (r0 + static_cast<int64_t>(part.runs.size()) >= (int64_t{1} << 31) ||
        c0 + static_cast<int64_t>(part.recs.size()) >= (int64_t{1} << 31))
        throw std::invalid_argument("tile schedule: more than 2^31 runs or ratings");
    for (int4 t : part.tiles)
        th.tiles.push_back(make_int4(t.x + e0, t.y, t.z + static_cast<int32_t>(r0), t.w + static_cast<int32_t>(c0)));
    th.users.insert(th.users.end(), part.users.begin(), part.users.end());
    th.streams.insert(th.streams.end(), part.streams.begin(), part.streams.end());
    th.runs.insert(th.runs.end(), part.runs.begin(), part.runs.end());
    th.recs.insert(th.recs.end(), part.recs.begin(), part.recs.end());
    th.pos.insert(th.pos.end(), part.pos.begin(), part.pos.end());
    th.split.insert(th.split.end(), part.split.begin(), part.split.end());
    th.lds = std::max(th.lds, part.lds);
}

// Strata (RS_EXCHANGE_ROTATE_Q): block b = this plan's ratings of items [ib[b], ib[b+1]) over all its users,
// tiled like a plan of its own (the item ids stay global: the kernel addresses the plan's whole Q).  Each
// block's user-CSR is filtered out of the plan's on pooled threads; positions map back to the plan's CSR.
void build_tile_strata(const rs_svd_plan* pl, int32_t grid0, bool want_pos, TileHost& th,
                       std::vector<int32_t>& block_tile, std::vector<int32_t>* block_split) {
    const std::vector<int32_t>& ib = pl->iblock_bounds;
    const int32_t nb = static_cast<int32_t>(ib.size()) - 1, nu = pl->n_users;
    const int32_t H = static_cast<int32_t>(pl->hot_items.size());
    std::vector<int32_t> blk(static_cast<size_t>(std::max(1, pl->n_items)), 0), hidx(blk.size(), -1);
    for (int32_t b = 0; b < nb; ++b)
        for (int32_t x = ib[b]; x < ib[b + 1]; ++x) blk[x] = b;
    for (int32_t h = 0; h < H; ++h) hidx[pl->hot_items[h]] = h;
    // a rating's stratum, and the Q row it trains: a hot item's rating goes to block mix32(user) mod nb and to
    // that block's copy of the item
    auto block_of = [&](int32_t u, int32_t item) {  // copy j of `copies`, blocks nb / copies apart from the natural one
        const int32_t h = hidx[item];
        if (h < 0) return blk[item];
        const int2 m = pl->hot_meta_h[h];
        const int32_t j = static_cast<int32_t>(mix32(static_cast<uint64_t>(u) * 0x9E3779B97F4A7C15ULL) % static_cast<uint32_t>(m.y));
        return (m.x + j * (nb / m.y)) % nb;
    };
    auto row_of = [&](int32_t b, int32_t item) { return hidx[item] < 0 ? item : pl->n_items + b * H + hidx[item]; };
    block_tile.assign(1, 0);
    if (block_split) block_split->assign(1, 0);
    const std::vector<int64_t>& rp = pl->h_rowptr;
    if (nb > 65535) throw std::invalid_argument("ROTATE_Q: at most 65535 item blocks");
    std::vector<uint16_t> rb(static_cast<size_t>(pl->nnz));  // every rating's block, one pass
    parallel_ranges(nu, 16, [&](int64_t u0, int64_t u1) {
        for (int64_t u = u0; u < u1; ++u)
            for (int64_t q = rp[u]; q < rp[u + 1]; ++q) rb[q] = static_cast<uint16_t>(block_of(static_cast<int32_t>(u), pl->h_cols[q]));
    });
    for (int32_t b = 0; b < nb; ++b) {
        rs_svd_plan sub;
        sub.n_users = nu;
        sub.n_items = pl->n_items + nb * H;  // the copies' rows
        sub.k = pl->k;
        sub.tile_waves = pl->tile_waves;
        sub.tile_claim = pl->tile_claim;
        sub.tile_user_lds = pl->tile_user_lds;
        sub.tile_target = pl->tile_target;
        sub.h_rowptr.assign(static_cast<size_t>(nu) + 1, 0);
        parallel_ranges(nu, 16, [&](int64_t u0, int64_t u1) {
            for (int64_t u = u0; u < u1; ++u) {
                int64_t c = 0;
                for (int64_t q = rp[u]; q < rp[u + 1]; ++q) c += rb[q] == b;
                sub.h_rowptr[u + 1] = c;
            }
        });
        for (int32_t u = 0; u < nu; ++u) sub.h_rowptr[u + 1] += sub.h_rowptr[u];
        sub.nnz = sub.h_rowptr[nu];
        sub.h_cols.resize(static_cast<size_t>(sub.nnz));
        sub.h_vals.resize(static_cast<size_t>(sub.nnz));
        std::vector<int64_t> orig(want_pos ? static_cast<size_t>(sub.nnz) : 0);
        parallel_ranges(nu, 16, [&](int64_t u0, int64_t u1) {
            for (int64_t u = u0; u < u1; ++u) {
                int64_t o = sub.h_rowptr[u];
                for (int64_t q = rp[u]; q < rp[u + 1]; ++q)
                    if (rb[q] == b) {
                        sub.h_cols[o] = row_of(b, pl->h_cols[q]);
                        sub.h_vals[o] = pl->h_vals[q];
                        if (want_pos) orig[o] = q;
                        ++o;
                    }
            }
        });
        const int32_t cap = pl->tile_run_cap > 0 ? pl->tile_run_cap : auto_run_cap(&sub, grid0, pl->tile_waves);
        TileHost part;
        build_tile_host(&sub, 0, nu, pl->tile_waves, tile_target_of(&sub, grid0, 0, nu), cap, want_pos, part);
        for (int64_t& x : part.pos) x = orig[x];
        append_tiles(th, std::move(part), b == 0);
        block_tile.push_back(static_cast<int32_t>(th.tiles.size()));
        if (block_split) block_split->push_back(static_cast<int32_t>(th.split.size()));
    }
}

void build_tile_blocks(const rs_svd_plan* pl, int32_t grid0, bool want_pos, TileHost& th,
                       std::vector<int32_t>& block_tile, std::vector<int32_t>& block_user,
                       std::vector<int32_t>* block_split = nullptr) {
    const std::vector<int64_t>& rp = pl->h_rowptr;
    if (!pl->iblock_bounds.empty()) {  // strata of a Q-rotation shard
        block_user = {0, pl->n_users};
        return build_tile_strata(pl, grid0, want_pos, th, block_tile, block_split);
    }
    if (!pl->ublock_bounds.empty()) {  // common bounds of the shards of a multi-GPU fit
        block_user = pl->ublock_bounds;
    } else {
        const int32_t nb = std::max(1, std::min(pl->tile_ublocks, std::max(1, pl->n_users)));
        block_user = user_block_bounds(rp.data(), pl->n_users, nb);
    }
    const int32_t nb = static_cast<int32_t>(block_user.size()) - 1;
    const int32_t cap = pl->tile_run_cap > 0 ? pl->tile_run_cap : auto_run_cap(pl, grid0, pl->tile_waves);
    block_tile.assign(1, 0);
    if (block_split) block_split->assign(1, 0);
    for (int32_t b = 0; b < nb; ++b) {
        const int32_t u0 = block_user[b], u1 = block_user[b + 1];
        TileHost part;
        build_tile_host(pl, u0, u1, pl->tile_waves, tile_target_of(pl, grid0, u0, u1), cap, want_pos, part);
        append_tiles(th, std::move(part), b == 0);
        block_tile.push_back(static_cast<int32_t>(th.tiles.size()));
        if (block_split) block_split->push_back(static_cast<int32_t>(th.split.size()));  // users ascend by block
    }
}

}  // namespace

int32_t tile_partials(const rs_svd_plan* pl) { return std::max(1, pl->tile_grid); }  // one per workgroup

int32_t tile_cap_in_use(const rs_svd_plan* pl) {
    ensure_host_csr(const_cast<rs_svd_plan*>(pl));
    if (pl->tile_run_cap > 0) return pl->tile_run_cap;
    const int32_t grid0 = tile_grid0(pl);
    const int32_t c = auto_run_cap(pl, grid0, pl->tile_waves);
    if (c > 0) return c;
    std::vector<int64_t> deg(std::max(1, pl->n_items), 0);  // uncut: the longest run is at most an item's degree
    for (int32_t x : pl->h_cols) deg[x]++;
    return static_cast<int32_t>(std::min<int64_t>(*std::max_element(deg.begin(), deg.end()), 1 << 30));
}

void tile_build(rs_svd_plan* pl) {
    if (pl->tile_rule == RS_TILE_RULE_FILL_DEVICE) {
        plan_sync_last(pl);
        if (!pl->coo_users.p) upload_coo_from_csr(pl);
        if (tile_build_device(pl)) return;
        pl->tile_rule = RS_TILE_RULE_LPT;  // the rule does not apply to this set: the host's default build
    }
    ensure_host_csr(pl);
    hipStream_t s = pl->ctx->stream;
    const int32_t grid0 = tile_grid0(pl);
    TileHost th;
    build_tile_blocks(pl, grid0, false, th, pl->t_block_tile, pl->t_block_user, &pl->t_block_split);
    plan_sync_last(pl);
    pl->n_tiles = static_cast<int32_t>(th.tiles.size());
    pl->t_n_runs = static_cast<int64_t>(th.runs.size());
    pl->t_n_users = static_cast<int64_t>(th.users.size());
    pl->tile_grid = std::max(1, std::min(grid0, pl->n_tiles));
    pl->tile_lds = std::max<size_t>(th.lds, 16);
    std::vector<int32_t> deg(static_cast<size_t>(std::max(1, pl->n_items)), 0);  // the hot-run damping's degrees
    for (int32_t c : pl->h_cols) deg[c]++;
    {  // cold runs: the header bit (sgd_plan.hpp kRunCold; the device build marks them the same way)
        const int64_t dcold = cold_degree_used(pl->cold_runs, pl->nnz, pl->n_items, pl->tile_grid, pl->tile_waves);
        pl->tile_cold = dcold > 0;
        if (dcold > 0)
            for (int2& r : th.runs)
                if (r.x >= 0 && r.x < pl->n_items && deg[r.x] < dcold) r.x |= kRunCold;
    }
    pl->t_tiles.alloc(std::max<size_t>(1, th.tiles.size()));
    pl->t_users.alloc(std::max<size_t>(1, th.users.size()));
    pl->t_streams.alloc(std::max<size_t>(1, th.streams.size()));
    pl->t_runs.alloc(std::max<size_t>(1, th.runs.size()));
    pl->t_recs.alloc(std::max<size_t>(1, th.recs.size()));
    {  // one pinned staging buffer for the five arrays (parallel copy in, then DMA): a pageable upload of
       // the ~12 MB of an ML-1M schedule took ~1 ms
        const size_t sz[5] = {th.tiles.size() * sizeof(int4), th.users.size() * sizeof(int2),
                              th.streams.size() * sizeof(int32_t), th.runs.size() * sizeof(int2),
                              th.recs.size() * sizeof(int2)};
        const void* src[5] = {th.tiles.data(), th.users.data(), th.streams.data(), th.runs.data(), th.recs.data()};
        void* dst[5] = {pl->t_tiles.p, pl->t_users.p, pl->t_streams.p, pl->t_runs.p, pl->t_recs.p};
        size_t off[6] = {0};
        for (int a = 0; a < 5; ++a) off[a + 1] = off[a] + (sz[a] + 255) / 256 * 256;
        // (the staging buffer lives as long as the ctx: schedules past kMaxPinnedStage, e.g. configs[4]'s
        // 1-GB shard schedule, upload from pageable memory instead of pinning that much for the ctx's life)
        constexpr size_t kMaxPinnedStage = size_t{256} << 20;
        char* stage = off[5] <= kMaxPinnedStage ? static_cast<char*>(pinned_staging(pl->ctx, off[5])) : nullptr;
        for (int a = 0; a < 5 && !stage; ++a)
            if (sz[a]) RS_HIP(hipMemcpyAsync(dst[a], src[a], sz[a], hipMemcpyHostToDevice, s));
        for (int a = 0; a < 5 && stage; ++a) {
            const char* from = static_cast<const char*>(src[a]);
            parallel_ranges(static_cast<int64_t>(sz[a]), 16, [&](int64_t b0, int64_t b1) {
                std::memcpy(stage + off[a] + b0, from + b0, static_cast<size_t>(b1 - b0));
            });
            if (sz[a]) RS_HIP(hipMemcpyAsync(dst[a], stage + off[a], sz[a], hipMemcpyHostToDevice, s));
        }
    }
    pl->t_n_split = static_cast<int32_t>(th.split.size());
    pl->t_split_rows.alloc(std::max<size_t>(1, th.split.size()));
    pl->t_split_rows.upload(th.split.data(), th.split.size(), s);
    pl->t_item_deg.alloc(deg.size());
    pl->t_item_deg.upload(deg.data(), deg.size(), s);
    pl->tile_damp = tile_damp_rule(*std::max_element(deg.begin(), deg.end()), pl->tile_grid, pl->tile_waves, pl->nnz);
    if (pl->t_n_split > 0 && pl->dPs.n != static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld) {
        pl->dPs.alloc(static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld);
        RS_HIP(hipMemsetAsync(pl->dPs.p, 0, pl->dPs.n * sizeof(float), s));
    }
    const size_t parts = static_cast<size_t>(tile_partials(pl));
    if (pl->partial.n < parts) pl->partial.alloc(parts);
    pl->tiles_built = true;
    RS_HIP(hipStreamSynchronize(s));  // host vectors die with this scope
}

void tile_order(rs_svd_plan* pl, int64_t* pos, int64_t* work_off, int32_t* n_works) {
    ensure_host_csr(pl);
    const int32_t grid0 = tile_grid0(pl);
    TileHost th;
    std::vector<int32_t> bt, bu;
    build_tile_blocks(pl, grid0, true, th, bt, bu);
    const size_t nw = th.tiles.size() * pl->tile_waves;
    if (n_works) *n_works = static_cast<int32_t>(nw);
    if (pos) std::copy(th.pos.begin(), th.pos.end(), pos);
    if (work_off) {  // stream s of tile t covers records [runs[first + st[s]].y, runs[first + st[s+1]].y)
        for (size_t t = 0; t < th.tiles.size(); ++t) {
            const int32_t* st = th.streams.data() + t * (pl->tile_waves + 1);
            for (int32_t s = 0; s <= pl->tile_waves; ++s) {
                if (s == pl->tile_waves && t + 1 < th.tiles.size()) break;
                work_off[t * pl->tile_waves + s] = th.tiles[t].w + th.runs[th.tiles[t].z + st[s]].y;
            }
        }
    }
}

struct TileRange {  // tiles [t0, t1) into dP rows of stride ldd (delta mode), grid workgroups
    int32_t t0, t1, ldd, grid;
    bool smooth = false;  // write the smoothed GlobalBias fold's sums (pl->gb_smooth; single-GPU epochs)
};

template <int E, int NW, int RQ, int CH, int DIAG = 0, bool DAMP = false, bool COLD = false>
static void tile_launch_t(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP, const TileRange& tr) {
    auto kern = svd_epoch_tile_kernel<E, NW, RQ, CH, DIAG, DAMP, COLD>;
    static bool attr = false;  // per instantiation
    if (!attr) {
        RS_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kTileLdsBudget)));
        attr = true;
    }
    const int32_t q_bytes = buffer_bytes32(pl->Q.n, sizeof(float), "item factor matrix");
    hipLaunchKernelGGL(kern, dim3(tr.grid), dim3(NW * 64), pl->tile_lds, s, pl->t_tiles.p + tr.t0, tr.t1 - tr.t0,
                       pl->t_users.p, pl->t_streams.p + static_cast<int64_t>(tr.t0) * (NW + 1), pl->t_runs.p,
                       pl->t_recs.p, pl->P.p, reinterpret_cast<int32_t*>(pl->Q.p), q_bytes, pl->gb.p, pl->partial.p,
                       pl->loss_part.n >= pl->partial.n ? pl->loss_part.p : nullptr, lr, reg, pl->fx(), dP, dP ? pl->uw.p : nullptr, pl->dPs.p, pl->k, pl->ld, tr.ldd, pl->trace.p,
                       pl->t_item_deg.p, buffer_bytes32(pl->t_item_deg.n, sizeof(int32_t), "item degrees"),
                       pl->damp_kconc > 0.f ? pl->damp_kconc
                                            : (pl->nnz > 0 ? static_cast<float>(static_cast<double>(tr.grid) * NW / static_cast<double>(pl->nnz)) : 0.f),
                       tr.smooth ? pl->gb_smooth.p : nullptr, std::log1p(-static_cast<double>(lr)));
}

// q_i rows in flight per wave (runs ahead): the ring's loads and the runs' atomics share the wave's
// in-order vmcnt, so a slot's load also waits for every atomic issued before it; the deeper the ring,
// the longer an atomic has to complete before a load behind it is needed.  Claimed runs (the default,
// pl->tile_claim > 0) take rings of 2 or 3 and chunks of 4 or 8 runs.
template <int E, int NW>
static void tile_launch_r(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP, const TileRange& tr) {
    constexpr int kMax = 60 / (2 * E);  // 15 at E = 2 (k <= 127), 6 at E = 5 (k <= 319), 3 at E = 8
    const int want = pl->tile_ring > 0 ? pl->tile_ring : 2;
    const bool claim = pl->tile_claim > 0;
    if constexpr (E == 2 && NW == 16) {  // diagnostics (RSGPU_TILE_DIAG, experiments only): bits drop
        static const int diag = std::getenv("RSGPU_TILE_DIAG") ? std::atoi(std::getenv("RSGPU_TILE_DIAG")) : 0;
        if ((diag & 48) && pl->trace.n < static_cast<size_t>(pl->tile_grid) * NW * 4) {
            pl->trace.alloc(static_cast<size_t>(pl->tile_grid) * NW * 4);
            RS_HIP(hipMemsetAsync(pl->trace.p, 0, pl->trace.n * 8, s));
        }
        switch (diag * (claim ? -1 : 1)) {  // 1 q atomics, 2 q loads, 4 p LDS atomics, 8 p LDS reads, 16 clocks
            case 1: return tile_launch_t<E, NW, 4, 0, 1>(pl, lr, reg, s, dP, tr);
            case 2: return tile_launch_t<E, NW, 4, 0, 2>(pl, lr, reg, s, dP, tr);
            case 3: return tile_launch_t<E, NW, 4, 0, 3>(pl, lr, reg, s, dP, tr);
            case 4: return tile_launch_t<E, NW, 4, 0, 4>(pl, lr, reg, s, dP, tr);
            case 16: return tile_launch_t<E, NW, 4, 0, 16>(pl, lr, reg, s, dP, tr);
            case -1: return tile_launch_t<E, NW, 2, 4, 1>(pl, lr, reg, s, dP, tr);
            case -3: return tile_launch_t<E, NW, 2, 4, 3>(pl, lr, reg, s, dP, tr);
            case -16: return tile_launch_t<E, NW, 2, 4, 16>(pl, lr, reg, s, dP, tr);
            case -32: return tile_launch_t<E, NW, 2, 4, 32>(pl, lr, reg, s, dP, tr);
            default: break;
        }
    }
    if (claim) {  // chunks of 8 runs and the 4-deep ring are instantiated for the bench's rows (E <= 2) only
        if constexpr (E <= 2) {
            // the ring must divide the chunk (static_assert in the kernel): a ring of 3 or more runs with
            // claims takes the 4-deep ring on chunks of 8
            if (want >= 3) return tile_launch_t<E, NW, 4, 8>(pl, lr, reg, s, dP, tr);
            if (pl->tile_claim >= 8) return tile_launch_t<E, NW, 2, 8>(pl, lr, reg, s, dP, tr);
        }
        // the default claims (4 runs, ring 2), with the hot-run damping where the schedule asks for it, or the cold
        // runs' stores where it marks them (a damped schedule's cold runs take the atomics)
        if (pl->tile_damp || pl->damp_kconc > 0.f) return tile_launch_t<E, NW, 2, 4, 0, true>(pl, lr, reg, s, dP, tr);
        if constexpr (NW == 16 || NW == 1) {  // (the library's waves; one wave: the exactness tests)
            if (pl->tile_cold) return tile_launch_t<E, NW, 2, 4, 0, false, true>(pl, lr, reg, s, dP, tr);
        }
        return tile_launch_t<E, NW, 2, 4>(pl, lr, reg, s, dP, tr);
    }
    // the host-dealt schedule (round 3; tile_claim = 0): rings 2 and 4, and 3 / 6 / 8 / 12 for E = 2
    if constexpr (E == 2) {
        if (want >= 12) return tile_launch_t<E, NW, 12, 0>(pl, lr, reg, s, dP, tr);
        if (want >= 8) return tile_launch_t<E, NW, 8, 0>(pl, lr, reg, s, dP, tr);
        if (want >= 6) return tile_launch_t<E, NW, 6, 0>(pl, lr, reg, s, dP, tr);
        if (want == 3) return tile_launch_t<E, NW, 3, 0>(pl, lr, reg, s, dP, tr);
    }
    if (want <= 3) return tile_launch_t<E, NW, 2, 0>(pl, lr, reg, s, dP, tr);
    if constexpr (kMax >= 4) {
        return tile_launch_t<E, NW, 4, 0>(pl, lr, reg, s, dP, tr);
    } else {
        return tile_launch_t<E, NW, kMax, 0>(pl, lr, reg, s, dP, tr);
    }
}

template <int E>
static void tile_launch_w(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP, const TileRange& tr) {
    switch (pl->tile_waves) {
        case 1: tile_launch_r<E, 1>(pl, lr, reg, s, dP, tr); break;
        case 2: tile_launch_r<E, 2>(pl, lr, reg, s, dP, tr); break;
        case 4: tile_launch_r<E, 4>(pl, lr, reg, s, dP, tr); break;
        case 8: tile_launch_r<E, 8>(pl, lr, reg, s, dP, tr); break;
        default: tile_launch_r<E, 16>(pl, lr, reg, s, dP, tr); break;
    }
}

static void tile_dispatch(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP, const TileRange& tr) {
    switch ((pl->k + 2 + 63) / 64) {  // registers per row: k factors + the two bias columns
        case 1: tile_launch_w<1>(pl, lr, reg, s, dP, tr); break;
        case 2: tile_launch_w<2>(pl, lr, reg, s, dP, tr); break;
        case 3: tile_launch_w<3>(pl, lr, reg, s, dP, tr); break;
        case 4: tile_launch_w<4>(pl, lr, reg, s, dP, tr); break;
        case 5: tile_launch_w<5>(pl, lr, reg, s, dP, tr); break;
        case 6: tile_launch_w<6>(pl, lr, reg, s, dP, tr); break;
        case 7: tile_launch_w<7>(pl, lr, reg, s, dP, tr); break;
        default: tile_launch_w<8>(pl, lr, reg, s, dP, tr); break;
    }
    RS_HIP(hipGetLastError());
}

static void tile_partials_fit(rs_svd_plan* pl, hipStream_t s) {
    if (pl->partial.n < static_cast<size_t>(tile_partials(pl))) {  // another schedule resized it
        plan_sync_last(pl);
        RS_HIP(hipStreamSynchronize(s));
        pl->partial.alloc(static_cast<size_t>(tile_partials(pl)));
    }
    if (pl->gb_smooth.n < 2 * pl->partial.n) {
        plan_sync_last(pl);
        RS_HIP(hipStreamSynchronize(s));
        pl->gb_smooth.alloc(2 * pl->partial.n);
    }
}

void tile_launch(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP) {
    if (!pl->tiles_built) tile_build(pl);
    pl->n_blocks = tile_partials(pl);
    tile_partials_fit(pl, s);
    if (pl->n_tiles == 0) {  // no ratings: the fold still reads its partials
        RS_HIP(hipMemsetAsync(pl->partial.p, 0, pl->partial.n * sizeof(double), s));
        RS_HIP(hipMemsetAsync(pl->gb_smooth.p, 0, pl->gb_smooth.n * sizeof(double), s));
        return;
    }
    // the single-GPU epoch (no dP) also writes the smoothed fold's sums; delta mode folds the mean of the moves
    TileRange tr{0, pl->n_tiles, pl->ld, pl->tile_grid};
    tr.smooth = dP == nullptr;
    tile_dispatch(pl, lr, reg, s, dP, tr);
}

int32_t tile_launch_range(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP, int32_t ldd,
                          int32_t t0, int32_t t1) {
    if (!pl->tiles_built) tile_build(pl);
    tile_partials_fit(pl, s);
    const int32_t grid = std::max(1, std::min(pl->tile_grid, t1 - t0));
    const int32_t parts = grid;  // one partial per workgroup
    if (t1 <= t0) {
        RS_HIP(hipMemsetAsync(pl->partial.p, 0, static_cast<size_t>(parts) * sizeof(double), s));
        return parts;
    }
    tile_dispatch(pl, lr, reg, s, dP, TileRange{t0, t1, ldd, grid});
    return parts;
}

}  // namespace rs

// Host-only diagnostic (no device): the tile schedule's host build for a user-CSR, timed.  Used to
// profile one-shot Fit's host share on the CPU and by the CPU tests.
extern "C" int rs_tile_schedule_host(int32_t n_users, int32_t n_items, const int64_t* rowptr, const int32_t* cols,
                                     const float* vals, int32_t n_factors, int32_t workgroups, int32_t waves,
                                     int32_t n_blocks, int32_t svdpp, int64_t* pos, int64_t* tile_off,
                                     int32_t* rank, int32_t* n_tiles, double* ms) {
    if (n_users < 0 || n_items < 0 || !rowptr || n_factors < 1 || n_factors > 510 || workgroups < 1 ||
        (waves != 1 && waves != 2 && waves != 4 && waves != 8 && waves != 16) || n_blocks == 0)
        return rs::set_error(nullptr, RS_ERR_INVALID, "bad tile schedule arguments");
    if (svdpp) return rs::set_error(nullptr, RS_ERR_UNSUPPORTED, "the SVD++ tile schedule was removed (round 3)");
    return rs_guard(nullptr, [&]() -> int {
        rs_svd_plan pl;
        pl.n_users = n_users;
        pl.n_items = n_items;
        pl.k = n_factors;
        pl.nnz = rowptr[n_users];
        pl.h_rowptr.assign(rowptr, rowptr + n_users + 1);
        pl.h_cols.assign(cols, cols + pl.nnz);
        pl.h_vals.assign(vals, vals + pl.nnz);
        pl.tile_waves = waves;
        if (n_blocks > 0) {
            pl.tile_ublocks = n_blocks;
        } else {  // -n item blocks of near-equal ratings: a ROTATE_Q shard's strata (no hot split)
            std::vector<int64_t> cum(static_cast<size_t>(n_items) + 1, 0);
            for (int64_t q = 0; q < pl.nnz; ++q) cum[cols[q] + 1]++;
            for (int32_t x = 0; x < n_items; ++x) cum[x + 1] += cum[x];
            pl.iblock_bounds = rs::user_block_bounds(cum.data(), n_items, -n_blocks);
        }
        const auto t0 = std::chrono::steady_clock::now();
        rs::TileHost th;
        std::vector<int32_t> bt, bu;
        rs::build_tile_blocks(&pl, workgroups, pos != nullptr, th, bt, bu);
        const auto t1 = std::chrono::steady_clock::now();
        if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (n_tiles) *n_tiles = static_cast<int32_t>(th.tiles.size());
        if (pos) std::copy(th.pos.begin(), th.pos.end(), pos);
        if (tile_off) {
            for (size_t t = 0; t < th.tiles.size(); ++t) tile_off[t] = th.tiles[t].w;
            tile_off[th.tiles.size()] = static_cast<int64_t>(th.recs.size());
        }
        if (rank) std::fill(rank, rank + th.recs.size(), 0);
        return RS_OK;
    });
}
