// sgd_ordered.hip -- the ORDERED SVD epoch (RS_SGD_ORDERED, north_star's "factor values within 1e-5 of
// the reference after one epoch"): core/svd.go:92-130 in the train-set order with the reference's update
// order and aliasing (p_u first, then q_i with the NEW p_u, Q1), every rating after the previous one.
//
// The serial dependence of that loop is narrower than it looks: rating t needs the rows rating t - d
// wrote only when it shares the user or the item, and the only state EVERY rating shares is the scalar
// GlobalBias chain gb <- gb - lr ((gb + b_u + b_i + p.q) - r) (svd.go:102-106), a first-order linear
// recurrence.  So the ratings are cut into batches in which no user and no item repeats, a batch's
// ratings run in parallel, and the chain runs as a scan (svd_ordered_batch_kernel below).  Also:
//   * the biases folded into the rows -- P row [p_0 .. p_{k-1}, b_u, 1], Q row [q_0 .. q_{k-1}, 1, b_i]
//     -- so p.q over all columns is the prediction minus gb, and the one update p <- a p - c q,
//     q <- a q - c p_new also performs svd.go:108-112 (the constant columns are held at 1);
//   * gb, the prediction and diff in float64 (the chain), the row arithmetic in float32.
// The result is the sequential epoch (no reordering), within float32 rounding of the fp64 restatement
// (tests/test_svd_gpu.py::test_ordered_*, 1e-5).  ML-1M shape, k = 100: 53.5 ms per epoch
// (1.87e7 updates/s, svd_ordered_group_kernel; the wave-per-rating form 75.4 ms); round 3's one-wave
// ring kernel took 222 ms, round 2's 16-lane group 515 ms.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "sgd_plan.hpp"

namespace rs {

namespace {

// DPP move of a double (both halves; lanes without a source read 0, rows outside row_mask keep 0)
template <int C, int RM>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(b), C, RM, 0xF, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(b >> 32), C, RM, 0xF, false);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}

__device__ __forceinline__ double readlane_f64(double x, int j) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(b), j);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(b >> 32), j);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}

}  // namespace

// One workgroup of NW waves walks the ratings in BATCHES: maximal runs of consecutive ratings (at most
// W = NW * R) in which no user and no item repeats (ordered_batches, on the host; 30.5 ratings on
// average on the ML-1M shape at W = 64).  Inside a batch the ratings touch disjoint rows, so their row
// updates commute; what they share is the GlobalBias chain gb <- gb - lr (gb + d_j) (svd.go:102-106,
// d_j = p.q + b_u + b_i - r_j), a first-order linear recurrence gb_{j+1} = a gb_j - lr d_j with a = 1 - lr:
//   1. wave w holds the rows of ratings w, w + NW, ... of batch c in registers (prefetched during batch
//      c - 1), except rows batch c - 1 rewrote, which it reads from the LDS copy that batch left;
//      it reduces d_j (biases folded into the rows) into LDS;
//   2. after one barrier every wave runs the chain as a lane-parallel scan of the affine maps (lane j:
//      gb after rating j, in six DPP steps), and issues the loads of batch c + 1's rows;
//   3. each wave applies svd.go:108-128 to its rows (p first, then q with the new p: Q1), stores them
//      and leaves a copy in LDS for batch c + 1.
// A row batch c + 1 loads from memory was last written by batch c - 1 or earlier; every wave drains its
// stores of batch c - 1 before batch c's first barrier, and batch c + 1's loads are issued after it.
// The result is the sequential epoch (the same rows meet the same updates in the same order); the
// GlobalBias values are the reference's recurrence evaluated in scan order (fp64; within 1e-15).
template <int H, int NW, int R>
__global__ __launch_bounds__(NW * 64) void svd_ordered_batch_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, const float* __restrict__ ratings,
    const int32_t* __restrict__ fwd, const int64_t* __restrict__ bstart, int64_t n_batches, float* P,
    int32_t p_bytes, float* Q, int32_t q_bytes, int32_t ld, int32_t kf, double* gb_io, int32_t epochs, float lr,
    float reg, uint64_t* prof /* diagnostics (RSGPU_ORDERED_PROF): wave 0's cycles per phase, or NULL */) {
#pragma clang fp contract(fast)
    constexpr int W = NW * R;
    static_assert(W <= 64, "a batch spans at most one wave's lanes");
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    __shared__ double sd[W];
    __shared__ f2 fp[W][H][64], fq[W][H][64];  // the rows batch c wrote, for batch c + 1
    const int lane = static_cast<int>(threadIdx.x & 63);
    const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(P, 0, p_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    int32_t coff[H];
    f2 amp[H], cmp[H], amq[H], cmq[H];
    const float a = 1.f - lr * reg;
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int32_t c = 128 * h + 2 * lane;
        coff[h] = c < ld ? 4 * c : kOutOfRange;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const bool kp = c + e == kf + 1, kq = c + e == kf;
            amp[h][e] = kp ? 1.f : a;
            cmp[h][e] = kp ? 0.f : 1.f;
            amq[h][e] = kq ? 1.f : a;
            cmq[h][e] = kq ? 0.f : 1.f;
        }
    }
    const double lrd = lr, al = 1.0 - lrd;
    // powers of a for the scan: a^(lane+1), a^(lane mod 16 + 1), a^(lane mod 32 + 1), a^1,2,4,8
    double pw1 = al, pw16 = al, pw32 = al;
    {
        double x = al;
        for (int j = 1; j < 64; ++j) {
            x *= al;
            pw1 = lane == j ? x : pw1;
            pw16 = (lane & 15) == j ? x : pw16;
            pw32 = (lane & 31) == j ? x : pw32;
        }
    }
    const double a2 = al * al, a4 = a2 * a2, a8 = a4 * a4;
    double gb = gb_io[0];
    auto off = [&](int32_t row, int h) {
        return static_cast<int32_t>(static_cast<uint32_t>(row) * static_cast<uint32_t>(ld * 4) + static_cast<uint32_t>(coff[h]));
    };
    const int64_t total = n_batches * static_cast<int64_t>(epochs);
    // A batch's ids live in VGPRs, lane x holding slot x (rating w + NW x): user, item, forward word (bits
    // 0-7: 1 + the slot of the previous batch that wrote this user's row, 0: none; bits 8-15 the same for
    // the item), rating.  Everything the loop reads from memory is a VECTOR load (vmcnt) issued a batch or
    // two ahead -- scalar loads would share lgkmcnt with the LDS traffic, and every LDS wait would then
    // wait for them too.  The arrays are padded by 64 entries past nnz; lanes x >= R repeat slot R - 1.
    struct Ids {
        int32_t u, i, f;
        float r;
    };
    const int xl = lane < R ? lane : R - 1;
    auto fetch_ids = [&](int64_t s0, Ids& d) {
        const int64_t e = s0 + w + NW * xl;
        d.u = users[e];
        d.i = items[e];
        d.f = fwd[e];
        d.r = ratings[e];
    };
    // batch bounds: lane 0 the start, lane 1 the end
    auto fetch_bounds = [&](int64_t b) { return bstart[b + (lane & 1)]; };
    auto s0_of = [](int64_t v) {
        return static_cast<int64_t>((static_cast<uint64_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), 0)) << 32) |
                                    __builtin_amdgcn_readlane(static_cast<uint32_t>(v), 0));
    };
    auto n_of = [](int64_t v) {
        return static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v), 1) - __builtin_amdgcn_readlane(static_cast<uint32_t>(v), 0));
    };
    auto next_b = [&](int64_t b) { return b + 1 == n_batches ? int64_t{0} : b + 1; };
    auto rl = [](int32_t v, int x) { return static_cast<int32_t>(__builtin_amdgcn_readlane(v, x)); };
    // rows of a batch from memory; a slot past n, or a row the previous batch rewrote (forwarded through
    // LDS instead), loads from row -1: past the buffer, 0
    auto load_rows = [&](const Ids& d, int32_t n, bool first, f2 (&p)[R][H], f2 (&q)[R][H]) {
#pragma unroll
        for (int x = 0; x < R; ++x) {
            if (w + NW * x >= n) continue;  // (uniform: slots past the batch are not touched at all)
            const int32_t f = rl(d.f, x);
            const int32_t ur = first || (f & 0xff) == 0 ? rl(d.u, x) : -1;
            const int32_t ir = first || (f & 0xff00) == 0 ? rl(d.i, x) : -1;
#pragma unroll
            for (int h = 0; h < H; ++h) {
                p[x][h] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rp, off(ur, h), 0, kSgdAux));
                q[x][h] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rq, off(ir, h), 0, kSgdAux));
            }
        }
    };
    uint64_t pc[6] = {0, 0, 0, 0, 0, 0}, tp = prof ? __builtin_amdgcn_s_memtime() : 0;
    auto ptick = [&](int ph) {
        if (prof) {
            const uint64_t tn = __builtin_amdgcn_s_memtime();
            pc[ph] += tn - tp;
            tp = tn;
        }
    };
    // prologue: batch 0's ids and rows, batch 1's ids, batch 2's bounds
    Ids cur, nxt;
    int64_t b1 = next_b(0), b2 = next_b(b1);
    const int64_t v0 = fetch_bounds(0), v1 = fetch_bounds(b1);
    int64_t vb = fetch_bounds(b2);  // bounds of batch t + 2
    int32_t n = n_of(v0), n1 = n_of(v1);
    fetch_ids(s0_of(v0), cur);
    fetch_ids(s0_of(v1), nxt);
    f2 p[R][H], q[R][H];
    load_rows(cur, n, true, p, q);
    for (int64_t t = 0; t < total; ++t) {
        // rows batch t - 1 rewrote: its LDS copies (the first batch of the launch has none)
        if (t > 0) {
#pragma unroll
            for (int x = 0; x < R; ++x) {
                if (w + NW * x >= n) continue;
                const int32_t f = rl(cur.f, x);
                const int32_t fu = (f & 0xff) - 1, fi = ((f >> 8) & 0xff) - 1;
                if (fu >= 0)
#pragma unroll
                    for (int h = 0; h < H; ++h) p[x][h] = fp[fu][h][lane];
                if (fi >= 0)
#pragma unroll
                    for (int h = 0; h < H; ++h) q[x][h] = fq[fi][h][lane];
            }
        }
        double dx[R];
#pragma unroll
        for (int x = 0; x < R; ++x) {
            dx[x] = 0.0;
            if (w + NW * x >= n) continue;
            f2 acc = p[x][0] * q[x][0];
#pragma unroll
            for (int h = 1; h < H; ++h) acc = __builtin_elementwise_fma(p[x][h], q[x][h], acc);
            const float sp = wave_sum(acc.x + acc.y);
            const float rx = __builtin_bit_cast(float, rl(__builtin_bit_cast(int32_t, cur.r), x));
            dx[x] = static_cast<double>(sp) - static_cast<double>(rx);  // svd.go:102 (minus gb)
            if (lane == 0) sd[w + NW * x] = dx[x];
        }
        ptick(0);
        __builtin_amdgcn_s_waitcnt(0);  // this wave's stores of batch t - 1 are done (see above)
        __syncthreads();
        ptick(1);
        double T = lane < n ? -lrd * sd[lane] : 0.0;
        // batch t + 1's rows (not rewritten by batch t), batch t + 2's ids, batch t + 3's bounds
        f2 pn[R][H], qn[R][H];
        load_rows(nxt, n1, false, pn, qn);
        Ids nn;
        fetch_ids(s0_of(vb), nn);
        const int32_t n2 = n_of(vb);
        b1 = b2;
        b2 = next_b(b2);
        const int64_t vbn = fetch_bounds(b2);
        // GlobalBias: T_j = sum_{i <= j} a^(j-i) (-lr d_i) by a Hillis-Steele scan (DPP row shifts inside
        // the 16-lane rows, then row_bcast:15 / row_bcast:31), G_j = a^(j+1) gb + T_j = gb after rating j
        T = __builtin_fma(al, dpp_f64<0x111, 0xF>(T), T);    // row_shr:1
        T = __builtin_fma(a2, dpp_f64<0x112, 0xF>(T), T);    // row_shr:2
        T = __builtin_fma(a4, dpp_f64<0x114, 0xF>(T), T);    // row_shr:4
        T = __builtin_fma(a8, dpp_f64<0x118, 0xF>(T), T);    // row_shr:8
        T = __builtin_fma(pw16, dpp_f64<0x142, 0xA>(T), T);  // row_bcast:15 into rows 1 and 3
        T = __builtin_fma(pw32, dpp_f64<0x143, 0xC>(T), T);  // row_bcast:31 into rows 2 and 3
        const double G = __builtin_fma(pw1, gb, T);
        ptick(2);
#pragma unroll
        for (int x = 0; x < R; ++x) {
            const int j = w + NW * x;
            if (j >= n) continue;
            const double g = j == 0 ? gb : readlane_f64(G, j > 0 ? j - 1 : 0);
            const float c = static_cast<float>(lrd * (g + dx[x]));  // lr diff
            const f2 cc = {c, c};
            const int32_t ur = rl(cur.u, x), ir = rl(cur.i, x);
#pragma unroll
            for (int h = 0; h < H; ++h) {  // svd.go:114-128: p first, then q with the NEW p (Q1)
                p[x][h] = __builtin_elementwise_fma(-q[x][h], cc * cmp[h], p[x][h] * amp[h]);
                q[x][h] = __builtin_elementwise_fma(-p[x][h], cc * cmq[h], q[x][h] * amq[h]);
                fp[j][h][lane] = p[x][h];
                fq[j][h][lane] = q[x][h];
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, p[x][h]), rp, off(ur, h), 0, 0);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, q[x][h]), rq, off(ir, h), 0, 0);
            }
        }
        gb = readlane_f64(G, n - 1);
        ptick(3);
        __syncthreads();  // the LDS copies are complete (the memory stores drain before the next barrier)
        ptick(4);
#pragma unroll
        for (int x = 0; x < R; ++x)
#pragma unroll
            for (int h = 0; h < H; ++h) {
                p[x][h] = pn[x][h];
                q[x][h] = qn[x][h];
            }
        cur = nxt;
        nxt = nn;
        n = n1;
        n1 = n2;
        vb = vbn;
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (threadIdx.x == 0) gb_io[0] = gb;
    if (prof && threadIdx.x == 0)
        for (int ph = 0; ph < 5; ++ph) prof[ph] = pc[ph];
}

// Rows of at most 128 floats (k <= 126): one 16-lane GROUP per rating instead of one wave, four ratings
// per wave instruction.  Lane t of a group holds columns [8t, 8t + 8) of a row as two float4; a slot's
// ids, forward word and rating are per-lane values (each lane of a group loads the same entry), the dot
// product is a 16-lane DPP sum, and a lane picks the GlobalBias before its rating from the scan by
// ds_bpermute.  Otherwise the batch protocol of svd_ordered_batch_kernel: rows prefetched a batch
// ahead, the previous batch's rows forwarded through LDS, one barrier before the scan and one after the
// LDS copies.  Slot j of a batch = 4 w + g + 4 NW x (wave w, group g, register slot x).
template <int NW, int R>
__global__ __launch_bounds__(NW * 64) void svd_ordered_group_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, const float* __restrict__ ratings,
    const int32_t* __restrict__ fwd, const int64_t* __restrict__ bstart, int64_t n_batches, float* P,
    int32_t p_bytes, float* Q, int32_t q_bytes, int32_t ld, int32_t kf, double* gb_io, int32_t epochs, float lr,
    float reg, uint64_t* prof) {
#pragma clang fp contract(fast)
    constexpr int GW = 4 * NW, W = GW * R;  // groups per workgroup, slots per batch
    static_assert(W <= 64, "a batch spans at most one wave's lanes (the scan)");
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __shared__ double sd[W];
    __shared__ f4 fp[W][16][2], fq[W][16][2];  // the rows batch c wrote, for batch c + 1
    const int lane = static_cast<int>(threadIdx.x & 63), grp = lane >> 4, tl = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(P, 0, p_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    int32_t coff[2];
    f4 amp[2], cmp[2], amq[2], cmq[2];
    const float a = 1.f - lr * reg;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int32_t c = 8 * tl + 4 * h;
        coff[h] = c < ld ? 4 * c : kOutOfRange;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool kp = c + e == kf + 1, kq = c + e == kf;
            amp[h][e] = kp ? 1.f : a;
            cmp[h][e] = kp ? 0.f : 1.f;
            amq[h][e] = kq ? 1.f : a;
            cmq[h][e] = kq ? 0.f : 1.f;
        }
    }
    const double lrd = lr, al = 1.0 - lrd;
    double pw1 = al, pw16 = al, pw32 = al;
    {
        double x = al;
        for (int j = 1; j < 64; ++j) {
            x *= al;
            pw1 = lane == j ? x : pw1;
            pw16 = (lane & 15) == j ? x : pw16;
            pw32 = (lane & 31) == j ? x : pw32;
        }
    }
    const double a2 = al * al, a4 = a2 * a2, a8 = a4 * a4;
    double gb = gb_io[0];
    auto off = [&](int32_t row, int h) {
        return static_cast<int32_t>(static_cast<uint32_t>(row) * static_cast<uint32_t>(ld * 4) + static_cast<uint32_t>(coff[h]));
    };
    auto slot = [&](int x) { return 4 * w + grp + GW * x; };  // this lane's slot (its group's rating)
    const int64_t total = n_batches * static_cast<int64_t>(epochs);
    struct Ids {
        int32_t u[R], i[R], f[R];
        float r[R];
    };
    auto fetch_ids = [&](int64_t s0, Ids& d) {  // vector loads (padded by 64 entries past nnz)
#pragma unroll
        for (int x = 0; x < R; ++x) {
            const int64_t e = s0 + slot(x);
            d.u[x] = users[e];
            d.i[x] = items[e];
            d.f[x] = fwd[e];
            d.r[x] = ratings[e];
        }
    };
    auto fetch_bounds = [&](int64_t b) { return bstart[b + (lane & 1)]; };
    auto s0_of = [](int64_t v) {
        return static_cast<int64_t>((static_cast<uint64_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), 0)) << 32) |
                                    __builtin_amdgcn_readlane(static_cast<uint32_t>(v), 0));
    };
    auto n_of = [](int64_t v) {
        return static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v), 1) - __builtin_amdgcn_readlane(static_cast<uint32_t>(v), 0));
    };
    auto next_b = [&](int64_t b) { return b + 1 == n_batches ? int64_t{0} : b + 1; };
    auto ld4 = [](__amdgpu_buffer_rsrc_t r, int32_t o) {
        return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, kSgdAux));
    };
    // rows of a batch from memory; a slot past n, or a row the previous batch rewrote (forwarded through
    // LDS instead), loads from row -1: past the buffer, 0
    auto load_rows = [&](const Ids& d, int32_t n, bool first, f4 (&p)[R][2], f4 (&q)[R][2]) {
#pragma unroll
        for (int x = 0; x < R; ++x) {
            if (4 * w + GW * x >= n) continue;  // (uniform: no group of this wave has a rating there)
            const bool ok = slot(x) < n;
            const int32_t ur = ok && (first || (d.f[x] & 0xff) == 0) ? d.u[x] : -1;
            const int32_t ir = ok && (first || (d.f[x] & 0xff00) == 0) ? d.i[x] : -1;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                p[x][h] = ld4(rp, off(ur, h));
                q[x][h] = ld4(rq, off(ir, h));
            }
        }
    };
    uint64_t pc[6] = {0, 0, 0, 0, 0, 0}, tp = prof ? __builtin_amdgcn_s_memtime() : 0;
    auto ptick = [&](int ph) {
        if (prof) {
            const uint64_t tn = __builtin_amdgcn_s_memtime();
            pc[ph] += tn - tp;
            tp = tn;
        }
    };
    Ids cur, nxt;
    int64_t b1 = next_b(0), b2 = next_b(b1);
    const int64_t v0 = fetch_bounds(0), v1 = fetch_bounds(b1);
    int64_t vb = fetch_bounds(b2);
    int32_t n = n_of(v0), n1 = n_of(v1);
    fetch_ids(s0_of(v0), cur);
    fetch_ids(s0_of(v1), nxt);
    f4 p[R][2], q[R][2];
    load_rows(cur, n, true, p, q);
    for (int64_t t = 0; t < total; ++t) {
        double dx[R];
#pragma unroll
        for (int x = 0; x < R; ++x) {
            dx[x] = 0.0;
            if (4 * w + GW * x >= n) continue;
            if (t > 0) {  // rows batch t - 1 rewrote: its LDS copies (the first batch has none)
                const int32_t fu = (cur.f[x] & 0xff) - 1, fi = ((cur.f[x] >> 8) & 0xff) - 1;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f4 a0 = fp[fu >= 0 ? fu : 0][tl][h], b0 = fq[fi >= 0 ? fi : 0][tl][h];
                    p[x][h] = fu >= 0 ? a0 : p[x][h];
                    q[x][h] = fi >= 0 ? b0 : q[x][h];
                }
            }
            const f4 m = p[x][0] * q[x][0] + p[x][1] * q[x][1];
            const float sp = group_sum<16>((m.x + m.y) + (m.z + m.w));
            dx[x] = static_cast<double>(sp) - static_cast<double>(cur.r[x]);  // svd.go:102 (minus gb)
            if (tl == 0 && slot(x) < n) sd[slot(x)] = dx[x];
        }
        ptick(0);
        __builtin_amdgcn_s_waitcnt(0);  // this wave's stores of batch t - 1 are done
        __syncthreads();
        ptick(1);
        double T = lane < n ? -lrd * sd[lane] : 0.0;
        f4 pn[R][2], qn[R][2];
        load_rows(nxt, n1, false, pn, qn);
        Ids nn;
        fetch_ids(s0_of(vb), nn);
        const int32_t n2 = n_of(vb);
        b1 = b2;
        b2 = next_b(b2);
        const int64_t vbn = fetch_bounds(b2);
        T = __builtin_fma(al, dpp_f64<0x111, 0xF>(T), T);    // row_shr:1
        T = __builtin_fma(a2, dpp_f64<0x112, 0xF>(T), T);    // row_shr:2
        T = __builtin_fma(a4, dpp_f64<0x114, 0xF>(T), T);    // row_shr:4
        T = __builtin_fma(a8, dpp_f64<0x118, 0xF>(T), T);    // row_shr:8
        T = __builtin_fma(pw16, dpp_f64<0x142, 0xA>(T), T);  // row_bcast:15 into rows 1 and 3
        T = __builtin_fma(pw32, dpp_f64<0x143, 0xC>(T), T);  // row_bcast:31 into rows 2 and 3
        const double G = __builtin_fma(pw1, gb, T);
        const uint64_t Gb = __builtin_bit_cast(uint64_t, G);
        ptick(2);
#pragma unroll
        for (int x = 0; x < R; ++x) {
            if (4 * w + GW * x >= n) continue;
            const int j = slot(x);
            const int src = 4 * (j > 0 ? j - 1 : 0);  // G of lane j - 1: gb before rating j
            const uint32_t glo = __builtin_amdgcn_ds_bpermute(src, static_cast<int32_t>(static_cast<uint32_t>(Gb)));
            const uint32_t ghi = __builtin_amdgcn_ds_bpermute(src, static_cast<int32_t>(static_cast<uint32_t>(Gb >> 32)));
            const double g = j == 0 ? gb : __builtin_bit_cast(double, (static_cast<uint64_t>(ghi) << 32) | glo);
            const float c = static_cast<float>(lrd * (g + dx[x]));  // lr diff
            const f4 cc = {c, c, c, c};
            const bool ok = j < n;
            const int32_t ur = ok ? cur.u[x] : -1, ir = ok ? cur.i[x] : -1;
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // svd.go:114-128: p first, then q with the NEW p (Q1)
                p[x][h] = __builtin_elementwise_fma(-q[x][h], cc * cmp[h], p[x][h] * amp[h]);
                q[x][h] = __builtin_elementwise_fma(-p[x][h], cc * cmq[h], q[x][h] * amq[h]);
                fp[j][tl][h] = p[x][h];
                fq[j][tl][h] = q[x][h];
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, p[x][h]), rp, off(ur, h), 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, q[x][h]), rq, off(ir, h), 0, 0);
            }
        }
        gb = readlane_f64(G, n - 1);
        ptick(3);
        __syncthreads();  // the LDS copies are complete (the memory stores drain before the next barrier)
        ptick(4);
#pragma unroll
        for (int x = 0; x < R; ++x)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                p[x][h] = pn[x][h];
                q[x][h] = qn[x][h];
            }
        cur = nxt;
        nxt = nn;
        n = n1;
        n1 = n2;
        vb = vbn;
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (threadIdx.x == 0) gb_io[0] = gb;
    if (prof && threadIdx.x == 0)
        for (int ph = 0; ph < 5; ++ph) prof[ph] = pc[ph];
}

// ORDERED epochs on the folded layout (rows of ld floats: P [p, b_u, 1], Q [q, 1, b_i]); users / items /
// ratings in train-set order, allocated for ordered_padded(nnz) entries.
int64_t ordered_padded(int64_t nnz) { return (nnz + 7) / 8 * 8 + 64; }

// Batches of the batched ORDERED kernel: a batch ends before the first rating whose user or item already
// occurs in it, or after wmax ratings.  start: n_batches + 1 offsets (the last one nnz).  fwd, per rating:
// 1 + the slot (position) in the previous batch that wrote its user's row (bits 0-7; 0: none) and its
// item's row (bits 8-15); batch 0's previous batch is the last one (the epochs repeat the sequence).
OrderedSchedule ordered_batches(const int32_t* users, const int32_t* items, int64_t nnz, int32_t n_users,
                                int32_t n_items, int32_t wmax) {
    OrderedSchedule o;
    o.start.reserve(static_cast<size_t>(nnz / 16 + 2));
    o.fwd.assign(static_cast<size_t>(nnz), 0);
    std::vector<int64_t> bu(static_cast<size_t>(std::max(1, n_users)), -2), bi(static_cast<size_t>(std::max(1, n_items)), -2);
    std::vector<int32_t> pu(bu.size(), 0), pi(bi.size(), 0);
    int64_t b = -1;
    int32_t n = wmax;
    for (int64_t t = 0; t < nnz; ++t) {
        const int32_t u = users[t], i = items[t];
        if (n == wmax || bu[u] == b || bi[i] == b) {
            o.start.push_back(t);
            ++b;
            n = 0;
        }
        o.fwd[t] = (bu[u] == b - 1 ? pu[u] + 1 : 0) | (bi[i] == b - 1 ? pi[i] + 1 : 0) << 8;
        bu[u] = bi[i] = b;
        pu[u] = pi[i] = n++;
    }
    o.start.push_back(nnz);
    const int64_t last = b;
    for (int64_t t = 0; t < (o.start.size() > 1 ? o.start[1] : 0); ++t) {
        const int32_t u = users[t], i = items[t];
        o.fwd[t] = (bu[u] == last ? pu[u] + 1 : 0) | (bi[i] == last ? pi[i] + 1 : 0) << 8;
    }
    return o;
}

int32_t ordered_wmax(int32_t ld) { return ld <= 256 ? 64 : 32; }

void ordered_epochs(const int32_t* users, const int32_t* items, const float* ratings, const int32_t* fwd,
                    int64_t nnz, const int64_t* bstart, int64_t n_batches, float* P, int64_t p_floats, float* Q,
                    int64_t q_floats, int32_t ld, int32_t kf, double* gb, int32_t epochs, float lr, float reg,
                    hipStream_t s) {
    if (nnz == 0 || epochs <= 0) return;
    if (p_floats * 4 >= (int64_t{1} << 31) || q_floats * 4 >= (int64_t{1} << 31))
        throw std::invalid_argument("ORDERED mode: factor matrices of 2 GiB or more");
    if (ld > 512) throw std::invalid_argument("ORDERED mode: rows of more than 512 floats");
    const int32_t pb = static_cast<int32_t>(p_floats * 4), qb = static_cast<int32_t>(q_floats * 4);
    // diagnostics: RSGPU_ORDERED_PROF=1 prints wave 0's cycles per phase of a batch
    const bool diag = [] { const char* e = std::getenv("RSGPU_ORDERED_PROF"); return e && std::atoi(e) != 0; }();
    DevBuf<uint64_t> dprof(diag ? 8 : 0);
    uint64_t* prof = diag ? dprof.p : nullptr;
    // rows of <= 128 floats: one 16-lane group per rating, RSGPU_ORDERED_GNW waves (16 default: 53.5 ms per
    // ML-1M epoch; 8: 54.2, 4: 65.1; 0 selects the wave-per-rating kernel, 75.4)
    const int gnw = [] { const char* e = std::getenv("RSGPU_ORDERED_GNW"); return e ? std::atoi(e) : 16; }();
    if (ld <= 128 && gnw > 0) {  // one 16-lane group per rating
        auto gk = [&](auto nw_c) {
            constexpr int NW = decltype(nw_c)::value;
            hipLaunchKernelGGL((svd_ordered_group_kernel<NW, 16 / NW>), dim3(1), dim3(NW * 64), 0, s, users, items,
                               ratings, fwd, bstart, n_batches, P, pb, Q, qb, ld, kf, gb, epochs, lr, reg, prof);
        };
        using std::integral_constant;
        if (gnw == 8) gk(integral_constant<int, 8>{});
        else if (gnw == 4) gk(integral_constant<int, 4>{});
        else gk(integral_constant<int, 16>{});
    } else {
    auto go = [&](auto h_c, auto nw_c) {
        constexpr int H = decltype(h_c)::value, NW = decltype(nw_c)::value;
        constexpr int W = H <= 2 ? 64 : 32;
        hipLaunchKernelGGL((svd_ordered_batch_kernel<H, NW, W / NW>), dim3(1), dim3(NW * 64), 0, s, users, items,
                           ratings, fwd, bstart, n_batches, P, pb, Q, qb, ld, kf, gb, epochs, lr, reg, prof);
    };
    using std::integral_constant;
    auto by_h = [&](auto nw_c) {
        if (ld <= 128) go(integral_constant<int, 1>{}, nw_c);
        else if (ld <= 256) go(integral_constant<int, 2>{}, nw_c);
        else go(integral_constant<int, 4>{}, nw_c);
    };
    by_h(integral_constant<int, 16>{});
    }
    RS_HIP(hipGetLastError());
    if (diag) {
        uint64_t h[8] = {0};
        RS_HIP(hipMemcpyAsync(h, prof, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        RS_HIP(hipStreamSynchronize(s));
        const double nb = static_cast<double>(n_batches) * epochs;
        std::fprintf(stderr, "ordered-prof %s NW=%d batches=%.0f cycles/batch: forward+dot %.0f drain+barrier1 %.0f "
                     "prefetch+scan %.0f update+store %.0f barrier2 %.0f\n", ld <= 128 && gnw > 0 ? "group" : "wave",
                     ld <= 128 && gnw > 0 ? gnw : 16, nb, h[0] / nb, h[1] / nb, h[2] / nb,
                     h[3] / nb, h[4] / nb);
    }
}

}  // namespace rs
