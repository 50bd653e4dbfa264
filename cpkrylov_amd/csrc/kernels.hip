// kernels.hip -- sparse kernels of the preconditioner apply and the Krylov operator
// (gfx950 / CDNA4, wave64).  All arithmetic is fp64 with FMA contraction disabled
// (-ffp-contract=off), and every row sum runs in increasing column order from 0, the
// accumulation order of MATLAB's sparse mtimes and column-oriented sparse mldivide, so the
// per-row results equal the CPU oracle bit for bit given equal inputs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <thread>
#include <tuple>
#include <cstdlib>
#include <cstring>

#include "dev.hpp"
#include "devutil.hpp"
#include "dist.hpp"
#include "spmv.hpp"
#include "xacc.hpp"

namespace cpk {

constexpr size_t kFactorPadEntries = 64;  // zero entries after fcol/fval/bcol/bval

void Ctx::ensure_partials(size_t count) {
    if (partials.n < count) partials.alloc(count);
    if (!counter.n) {
        counter.alloc(kTicketWords);
        CPK_HIP(hipMemset(counter.p, 0, counter.bytes()));
    }
    if (exact()) ensure_xacc(4);
}

void Ctx::ensure_xacc(size_t nsums) {
    if (xsub.n < (size_t)kXSub * kXW * nsums) {
        xsub.alloc((size_t)kXSub * kXW * nsums);
        CPK_HIP(hipMemset(xsub.p, 0, xsub.bytes()));  // the launches leave them zero
    }
    if (dist() && xred.n < (size_t)kXW * nsums) xred.alloc((size_t)kXW * nsums);
}

// the rounded global sums of the exact digits: out[j] = xround(dig[j]) on every rank
__global__ void xround_kernel(int64_t *dig, int nv, double *out) {
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nv; j += gridDim.x * blockDim.x)
        out[j] = xround(dig + (size_t)j * kXW);  // normalises the (allreduced, dead) digits in place
}

void allreduce_red(Ctx &c, int nv) {
    if (!c.exact()) {
        c.comm->allreduce_sum(c.red.p, (size_t)nv, c.stream);
        return;
    }
    if ((size_t)nv > c.red.n || (size_t)nv * kXW > c.xred.n)
        throw Error(CPK_ERR_UNSUPPORTED, "exact reduction wider than its buffers");
    c.comm->allreduce_sum_i64(c.xred.p, (size_t)nv * kXW, c.stream);
    hipLaunchKernelGGL(xround_kernel, dim3(1), dim3(256), 0, c.stream, c.xred.p, nv, c.red.p);
    CPK_HIP(hipGetLastError());
}

// ---- device matrix layout -------------------------------------------------------------------
void make_dmat(const HCsr &a, DMat &d) {
    static std::atomic<uint64_t> gen{1};
    d.gen = gen++;
    if (a.nnz() > (int64_t)UINT32_MAX) throw Error(CPK_ERR_UNSUPPORTED, "more than 2^32 nonzeros in one matrix");
    d.nrows = a.nrows, d.ncols = a.ncols, d.nnz = a.nnz();
    std::vector<uint32_t> ptr(a.ptr.begin(), a.ptr.end());
    std::vector<int32_t> blk{0};
    int64_t r0 = 0;
    for (int64_t r = 0; r < a.nrows; r++) {
        int64_t rows = r - r0, ents = a.ptr[r + 1] - a.ptr[r0];
        if (rows > 0 && (rows >= kSpmvMaxRows || ents > kSpmvCap)) {
            blk.push_back((int32_t)r);
            r0 = r;
        }
    }
    blk.push_back((int32_t)a.nrows);  // an empty matrix keeps one (empty) block: every launch has a grid
    d.nblk = (int64_t)blk.size() - 1;
    d.ptr.upload(ptr);
    d.col.upload(a.ind);
    d.val.upload(a.val);
    d.blk.upload(blk);
    d.is_diag = is_diagonal(a);
}

// ---- factor layout ---------------------------------------------------------------------------
// Row entries are stored in the accumulation order of the reference solve on the factor the
// caller exports: forward rows by ascending key of the column, backward rows (columns of L)
// by descending key of the row.  key[q] is the pre-relabel index of relabelled row q (so a
// relabelled factor still sums in the exported factor's order); extra[q] are backward entries
// of row q that refer to rows outside this factor (distributed separators).
// entries per LDS round trip in the upper-round level loop, per direction: the forward rows
// carry tens of in-block terms, the backward ones few (stamps build, profiles/r03_upper_ch_v17.txt:
// 8 vs 4 per chunk, forward levels -7 % / -11 % in rounds 1 / 2, backward +14 % / +17 %)
#ifndef CPK_UPPER_CH_FWD
#define CPK_UPPER_CH_FWD 8
#endif
#ifndef CPK_UPPER_CH_BWD
#define CPK_UPPER_CH_BWD 4
#endif
// round 0 on the dataflow loop: 0 never, 1 both directions (default), 2 forward only; terms per
// iteration.  A/B at S10 (profiles/r04_r0_dataflow_ab_v7.txt): 2 terms per iteration take the
// round-0 forward sweep 188 -> 170-178 us and the fused residual forward 260 -> 251-256 us; the
// backward 180-182 -> 177 us once a lane walks a mask of its rows (4 terms spill)
#ifndef CPK_R0_DATAFLOW
#define CPK_R0_DATAFLOW 1
#endif
#ifndef CPK_R0_DF_CH_FWD
#define CPK_R0_DF_CH_FWD 2
#endif
#ifndef CPK_R0_DF_CH_BWD
#define CPK_R0_DF_CH_BWD 1  // backward rows of round 0 carry ~2 in-block terms: 1 per iteration
#endif                      // (profiles/r04_r0_bwd_ch_ab_v15.txt: 3 / 4 terms slower, 1 forward slower)
// the dataflow level loop (levels_dataflow) where mark_dataflow picks it; terms per iteration;
// the modelled cost of one of its trips relative to a level-loop trip: 2.0 for the first loop
// (8 terms, a row-switch loop, short-circuit flag reads), 1.0 since the mask walk, the
// branch-free ready prefix and 4 / 2 terms (profiles/r04_dataflow_alpha_ab_v11.txt: S10 +0.4 %,
// P = 8 rank -1.2 %, the +-64 window 324 -> 357 it/s)
constexpr double kDataflowTripCost = 1.0;
// the column sweep (levels_colsweep): blocks of at most 256 rows (4 per lane).  The choice
// against the other loops is made in cycles, fitted on the stamps build over every upper block of
// the +-64 window with the column sweep forced on and off (tools/upper_cycles.py BLOCKS=,
// profiles/r05_colsweep_calibration.txt): cycles per step at 1 / 2 / 3 / 4 rows per lane, without
// and with drains, and per drain trip; a level-loop trip ~290 cycles, a dataflow trip ~270
// forward / ~190 backward (3 and 4 rows per lane: extrapolated, no such block measured)
constexpr int kColsweepMaxRows = 4 * 64;
constexpr double kColsweepStepCycles[4] = {220.0, 257.0, 340.0, 420.0};
constexpr double kColsweepStepDrainCycles[4] = {297.0, 353.0, 430.0, 500.0};
// the column sweep's staged columns (DFactor::ucode): an in-block entry holds its column's step |
// the run of outside entries behind it (up to the next in-block entry or the row's end) << 8, an
// outside entry kCsOut
constexpr int kCsOut = 0x8000, kCsStep = 0x80ff, kCsRunMax = 127;
constexpr double kColsweepDrainCycles[4] = {261.0, 617.0, 800.0, 1000.0};  // a drain trip (four terms a row)
constexpr double kLevelTripCycles = 290.0, kDataflowTripCycles[2] = {272.0, 190.0};
#ifndef CPK_UPPER_DATAFLOW
#define CPK_UPPER_DATAFLOW 1
#endif
// (per direction; the +-64 window, profiles/r04_dataflow_ch_ab_v10.txt: forward 8 / 4 / 2 terms
// 0.767 / 0.732 / 0.900 ms per sweep, backward 0.690 / 0.574 / 0.536)
#ifndef CPK_DF_CH_FWD
#define CPK_DF_CH_FWD 4
#endif
#ifndef CPK_DF_CH_BWD
#define CPK_DF_CH_BWD 2
#endif
#define CPK_DF_CH(bwd) ((bwd) ? CPK_DF_CH_BWD : CPK_DF_CH_FWD)
// Level loop or dataflow loop (levels_dataflow) for an upper-round block's levels, chosen per
// block and direction on the host from a model of each loop's dependent LDS round trips:
//   level loop (sweep_levels, one wave): per level and pass of 64 rows, one trip for the rows'
//     bounds and one pair per chunk of CPK_UPPER_CH terms of the level's longest row;
//   dataflow loop: its lock-step schedule simulated exactly (a row's terms taken CPK_DF_CH at a
//     time once their columns were finished in an earlier iteration), a pair of trips per
//     iteration plus one per row switch.
// The dataflow loop wins on dense chains (a separator clique: a level per row, tens of terms
// each) and loses on wide shallow blocks, where a lane's rows wait on each other in sequence.
// The choice is bits 30 (forward) / 29 (backward) of the block record's l1 (kernels mask them).
namespace {
int64_t level_trips(const std::vector<int32_t> &lvl_bounds, const std::vector<int> &nterm, int ch) {
    int64_t trips = 0;
    for (size_t l = 0; l + 1 < lvl_bounds.size(); l++) {
        for (int a = lvl_bounds[l]; a < lvl_bounds[l + 1]; a += kWave) {
            int mx = 0;
            for (int k = a; k < std::min(a + kWave, (int)lvl_bounds[l + 1]); k++) mx = std::max(mx, nterm[k]);
            trips += 1 + 2 * ((mx + ch - 1) / ch);
        }
    }
    return trips;
}
// terms[k]: the row's loop terms (after the folded outside prefix), -1 for an outside term;
// order[i]: the i-th row solved (lane i % 64); returns trips, or `stop` once it exceeds it
int64_t dataflow_trips(const std::vector<std::vector<int>> &terms, bool bwd, int ch, int64_t stop) {
    const int nr = (int)terms.size();
    std::vector<int64_t> done(nr, INT64_MAX);
    struct Lane { int i, e; };
    std::vector<Lane> L(kWave);
    for (int l = 0; l < kWave; l++) L[l] = {l, 0};
    auto row = [&](int i) { return bwd ? nr - 1 - i : i; };
    int64_t trips = 1;
    for (int64_t it = 0;; it++) {
        bool any = false;
        int switches = 0;
        for (int l = 0; l < kWave; l++) {
            Lane &z = L[l];
            if (z.i >= nr) continue;
            any = true;
            const std::vector<int> &t = terms[row(z.i)];
            for (int j = 0; j < ch && z.e < (int)t.size(); j++) {
                const int c = t[z.e];
                if (c >= 0 && done[c] >= it) break;
                z.e++;
            }
            int sw = 0;
            while (z.i < nr && z.e >= (int)terms[row(z.i)].size()) {
                done[row(z.i)] = it;
                z.i += kWave, z.e = 0, sw++;
            }
            switches = std::max(switches, sw);
        }
        if (!any) return trips;
        trips += 2 + switches;
        if (trips > stop) return trips;
    }
}
}  // namespace

// the upper rounds' row data for the block kernels (DFactor::ufold, [2 (row - urow0) + bwd]):
//   fold: the leading outside-term count of each row and direction, the entries before the first
//     one inside the row's block -- what fold_prefix finds by testing each column (fold_known).
//     Capped at INT16_MAX (a shorter fold is still exact: the loops take the rest against the
//     1.0 slot);
//   step: the row's position in its block by ascending key (forward) / descending key (backward)
//     -- the entry order of every row, so an order in which each row's terms are met in its own
//     order (levels_colsweep).
template <class Key>
static std::vector<int16_t> build_ufold(DFactor &d, const std::vector<int32_t> &meta, const std::vector<int64_t> &round_ptr,
                        const std::vector<uint32_t> &fptr, const std::vector<int32_t> &fcol,
                        const std::vector<uint32_t> &bptr, const std::vector<int32_t> &bcol, const Key &key) {
    d.ufold.release();
    d.ustep.release();
    d.ucode[0].release(), d.ucode[1].release();
    d.urow0 = 0, d.ucode0[0] = d.ucode0[1] = 0;
    if (round_ptr.size() < 3) return {};
    const int64_t ub0 = round_ptr[1], ub1 = round_ptr.back();
    int64_t lo = INT64_MAX, hi = 0;
    for (int64_t b = ub0; b < ub1; b++) lo = std::min<int64_t>(lo, meta[(size_t)b * 8]), hi = std::max<int64_t>(hi, meta[(size_t)b * 8 + 1]);
    if (lo >= hi) return {};
    std::vector<int16_t> uf((size_t)(2 * (hi - lo)), 0), us((size_t)(2 * (hi - lo)), 0);
    std::vector<int16_t> code[2] = {std::vector<int16_t>((size_t)(fptr[hi] - fptr[lo]), 0),
                                    std::vector<int16_t>((size_t)(bptr[hi] - bptr[lo]), 0)};
    parallel_for(ub1 - ub0, [&](int64_t a, int64_t z) {
        std::vector<std::pair<int64_t, int32_t>> order;
        for (int64_t b = ub0 + a; b < ub0 + z; b++) {
            const int32_t r0 = meta[(size_t)b * 8], r1 = meta[(size_t)b * 8 + 1];
            for (int32_t i = r0; i < r1; i++)
                for (int dir = 0; dir < 2; dir++) {
                    const std::vector<uint32_t> &ptr = dir ? bptr : fptr;
                    const std::vector<int32_t> &col = dir ? bcol : fcol;
                    uint32_t e = ptr[i];
                    while (e < ptr[i + 1] && !(col[e] >= r0 && col[e] < r1)) e++;
                    uf[(size_t)(2 * (i - lo) + dir)] = (int16_t)std::min<uint32_t>(e - ptr[i], INT16_MAX);
                }
            if (r1 - r0 > INT16_MAX) continue;
            order.clear();
            for (int32_t i = r0; i < r1; i++) order.push_back({key(i), i});
            std::sort(order.begin(), order.end());
            const int32_t nr = r1 - r0;
            for (int32_t t = 0; t < nr; t++) {
                const int32_t i = order[(size_t)t].second;
                us[(size_t)(2 * (i - lo))] = (int16_t)t, us[(size_t)(2 * (i - lo) + 1)] = (int16_t)(nr - 1 - t);
            }
            if (nr > kColsweepMaxRows) continue;
            // staged columns of the column sweep: in-block steps with the outside run behind each
            for (int32_t i = r0; i < r1; i++)
                for (int dir = 0; dir < 2; dir++) {
                    const std::vector<uint32_t> &ptr = dir ? bptr : fptr;
                    const std::vector<int32_t> &col = dir ? bcol : fcol;
                    int16_t *cd = code[dir].data() - (dir ? bptr[lo] : fptr[lo]);
                    int64_t last = -1;
                    int run = 0;
                    for (uint32_t e = ptr[i]; e < ptr[i + 1]; e++) {
                        const int32_t c = col[e];
                        if (c >= r0 && c < r1) {
                            if (last >= 0) cd[last] = (int16_t)(cd[last] | (std::min(run, kCsRunMax) << 8));
                            cd[e] = us[(size_t)(2 * (c - lo) + dir)], last = e, run = 0;
                        } else {
                            cd[e] = (int16_t)kCsOut, run += last >= 0;
                        }
                    }
                    if (last >= 0) cd[last] = (int16_t)(cd[last] | (std::min(run, kCsRunMax) << 8));
                }
        }
    }, 64);
    d.urow0 = (int32_t)lo;
    d.ufold.upload(uf);
    d.ustep.upload(us);
    d.ucode[0].upload(code[0]), d.ucode[1].upload(code[1]);
    d.ucode0[0] = fptr[lo], d.ucode0[1] = bptr[lo];
    return us;
}
void mark_dataflow(std::vector<int32_t> &meta, const std::vector<int64_t> &round_ptr, const std::vector<uint32_t> &fptr,
                   const std::vector<int32_t> &fcol, const std::vector<uint32_t> &bptr, const std::vector<int32_t> &bcol,
                   int mode, int cs_mode, const std::vector<int16_t> &ustep, int64_t urow0,
                   std::vector<int64_t> *model) {
    if (model) model->clear();
    if (round_ptr.size() < 3) return;
    const int64_t b0 = round_ptr[1], b1 = round_ptr.back();  // the upper rounds
    // per block and direction: nr, level trips, dataflow trips, outside terms behind in-block
    // ones, column sweep valid, flags chosen (cpk_debug_block_model: the loops' cost model)
    if (model) model->assign((size_t)(b1 - b0) * 2 * kBlockModelW, -1);
    const double alpha = kDataflowTripCost;
    const bool df_on = CPK_UPPER_DATAFLOW && mode != 1;
    parallel_for(b1 - b0, [&](int64_t lo, int64_t hi) {
        std::vector<int32_t> lb;
        std::vector<int> nterm;
        std::vector<std::vector<int>> terms;
        for (int64_t b = b0 + lo; b < b0 + hi; b++) {
            int32_t *m = &meta[(size_t)b * 8];
            const int r0 = m[0], r1 = m[1], nr = r1 - r0;
            for (int dir = 0; dir < 2; dir++) {
                const std::vector<uint32_t> &ptr = dir ? bptr : fptr;
                const std::vector<int32_t> &col = dir ? bcol : fcol;
                terms.assign((size_t)nr, {});
                nterm.assign((size_t)nr, 0);
                for (int k = 0; k < nr; k++) {
                    uint32_t e = ptr[r0 + k];
                    const uint32_t e1 = ptr[r0 + k + 1];
                    while (e < e1 && !(col[e] >= r0 && col[e] < r1)) e++;  // fold_prefix's leading outside terms
                    for (; e < e1; e++) terms[k].push_back(col[e] >= r0 && col[e] < r1 ? col[e] - r0 : -1);
                    nterm[k] = (int)terms[k].size();
                }
                // level bounds of the block (rows are contiguous by level): from the row dependencies
                // the kernel's level array describes -- recomputed here as the longest path
                std::vector<int> lev((size_t)nr, 0);
                int nlev = 0;
                for (int q = 0; q < nr; q++) {
                    const int k = dir ? nr - 1 - q : q;
                    for (int c : terms[k]) if (c >= 0) lev[k] = std::max(lev[k], lev[c] + 1);
                    nlev = std::max(nlev, lev[k] + 1);
                }
                // rows per level (the kernel walks each level's rows in passes of 64)
                std::vector<int> cnt((size_t)nlev, 0), mx((size_t)nlev, 0);
                lb.assign((size_t)nlev + 1, 0);
                std::vector<int> byl((size_t)nr);
                for (int k = 0; k < nr; k++) cnt[lev[k]]++;
                for (int l = 0; l < nlev; l++) lb[l + 1] = lb[l] + cnt[l];
                {
                    std::vector<int> pos(lb.begin(), lb.end() - 1);
                    for (int k = 0; k < nr; k++) byl[pos[lev[k]]++] = nterm[k];
                }
                const int64_t lt = level_trips(lb, byl, dir ? CPK_UPPER_CH_BWD : CPK_UPPER_CH_FWD);
                const int64_t dt = df_on ? dataflow_trips(terms, dir == 1, CPK_DF_CH(dir == 1), (int64_t)(4 * lt) + 8)
                                         : INT64_MAX;
                const bool df = df_on && (mode == 2 || alpha * (double)dt < (double)lt);
                // the column sweep (levels_colsweep): one step per row, its cost per step growing
                // with the rows each lane holds; outside terms behind in-block ones add a pass each
                // valid only if every row meets its in-block terms at increasing steps, all before
                // its own (the steps follow the entries' key order; checked, not assumed)
                // valid only if the kernel's schedule takes every term of every row before the
                // row's own step, one term per step: an in-block term at its column's step, an
                // outside term at the first step after the row's previous term (the steps follow
                // the entries' key order; checked, not assumed)
                // Without drains (one term per step) it needs every outside term to find a free
                // step before the row's next in-block term and its own step; with drains it needs
                // the in-block terms at increasing steps before the row's own, and costs a drain
                // trip per step and outside term behind that step's in-block ones (the longest run)
                bool cs = false, drain = false, cs_valid = cs_mode != 1 && nr <= kColsweepMaxRows && !ustep.empty();
                auto step = [&](int k) { return (int)ustep[(size_t)(2 * (r0 + k - urow0) + dir)]; };
                std::vector<int> run(cs_valid ? (size_t)nr : 0, 0);  // per step: longest outside run behind it
                int maxrun = 0;
                for (int k = 0; k < nr && cs_valid; k++) {
                    int t = 0, prev = -1, out = 0;  // t: the first step free for the row's next term
                    for (int c : terms[k]) {
                        if (c < 0) {
                            t++, out++;
                            if (prev >= 0) run[(size_t)prev] = std::max(run[(size_t)prev], out);
                            maxrun = std::max(maxrun, out);
                        } else {
                            cs_valid = cs_valid && step(c) > prev && step(c) < step(k);
                            drain = drain || step(c) < t;
                            t = step(c) + 1, prev = step(c), out = 0;
                        }
                    }
                    drain = drain || t > step(k);
                }
                cs_valid = cs_valid && !(drain && maxrun > 127);  // kCsRunMax: a run's length in its staged column
                if (cs_valid) {
                    const int rpl = std::min((nr + kWave - 1) / kWave, 4);
                    int64_t trips = 0;  // drain trips: four terms of every row's run per trip
                    if (drain)
                        for (int x : run) trips += (x + 3) / 4;
                    const double ct = (double)nr * (drain ? kColsweepStepDrainCycles : kColsweepStepCycles)[rpl - 1] +
                                      (double)trips * kColsweepDrainCycles[rpl - 1];
                    const double base = df ? kDataflowTripCycles[dir] * (double)dt : kLevelTripCycles * (double)lt;
                    cs = cs_mode == 2 || ct < base;
                }
                if (cs) m[3] |= (dir ? kMetaCsBwd : kMetaCsFwd) | (drain ? (dir ? kMetaCoBwd : kMetaCoFwd) : 0);
                else if (df) m[3] |= dir ? kMetaDfBwd : kMetaDfFwd;
                if (model) {
                    int64_t *o = &(*model)[(size_t)(((b - b0) * 2 + dir) * kBlockModelW)];
                    int64_t outs = 0;
                    for (int k = 0; k < nr; k++)
                        for (int c : terms[k]) outs += c < 0;
                    o[0] = b, o[1] = dir, o[2] = nr, o[3] = lt, o[4] = df_on ? dt : -1, o[5] = outs, o[6] = cs_valid,
                    o[7] = cs ? (drain ? 3 : 2) : (df ? 1 : 0);
                }
            }
        }
    }, 4);
}

static void build_chain(DFactor &d, const std::vector<int32_t> &meta, const std::vector<uint32_t> &fptr,
                        const std::vector<int32_t> &fcol, const std::vector<uint32_t> &bptr,
                        const std::vector<int32_t> &bcol);
constexpr int64_t kInsertionSortMax = 32;  // rows up to this long sort by insertion (keys are distinct)
void make_dfactor(const Factor &f, const Schedule &s, DFactor &d, const std::vector<int64_t> *key,
                  const std::vector<std::vector<BwdExtra>> *extra, std::vector<int32_t> *fsrc,
                  std::vector<int32_t> *bsrc) {
    const int64_t N = f.N;
    SubClock clk;
    auto K = [&](int64_t q) { return key ? (*key)[q] : q; };
    int64_t nextra = 0;
    if (extra)
        for (const auto &e : *extra) nextra += (int64_t)e.size();
    if (extra && bsrc) throw Error(CPK_ERR_UNSUPPORTED, "internal: entry sources with extra backward entries");
    // structure-only factor (no D): values come from the device numeric phase.  Not f.Lx: a
    // numeric factor without off-diagonal entries has an empty Lx but a valid D
    const bool vals = (int64_t)f.D.size() == f.N;
    d.N = N;
    d.nnz = (int64_t)f.Li.size() + nextra;
    if (d.nnz > (int64_t)INT32_MAX) throw Error(CPK_ERR_UNSUPPORTED, "factor has more than 2^31 entries");
    // forward rows: transpose of the CSC, then each row ordered by the key of its columns;
    // fidx[q] = the CSC slot of forward entry q
    std::vector<uint32_t> fptr(N + 1, 0);
    const int64_t nf = (int64_t)f.Li.size();
    std::vector<int32_t> fcol, fidx, bcol, bidx;
    {
        // the large index arrays are zero-filled (first touch of fresh pages) on threads of their
        // own; the padding below appends without a reallocation
        std::vector<std::thread> al;
        al.emplace_back([&] { fcol.reserve((size_t)nf + kFactorPadEntries), fcol.resize(nf); });
        al.emplace_back([&] { bcol.reserve((size_t)d.nnz + kFactorPadEntries), bcol.resize(d.nnz); });
        al.emplace_back([&] { bidx.resize(bsrc ? d.nnz : 0); });
        fidx.resize(nf);
        for (auto &x : al) x.join();
    }
    {
        transpose_pattern(N, f.Lp.data(), f.Li.data(), fptr.data(), fcol.data(), fidx.data());
        if (key)
            parallel_for(N, [&](int64_t lo, int64_t hi) {  // rows sort independently (keys distinct)
                std::vector<std::pair<int64_t, std::pair<int32_t, int32_t>>> row;
                for (int64_t i = lo; i < hi; i++) {
                    const uint32_t a = fptr[i], z = fptr[i + 1];
                    if (z - a <= kInsertionSortMax) {  // short rows: insertion sort in place
                        for (uint32_t q = a + 1; q < z; q++) {
                            const int32_t c = fcol[q], x = fidx[q];
                            const int64_t kc = K(c);
                            uint32_t r = q;
                            for (; r > a && K(fcol[r - 1]) > kc; r--) fcol[r] = fcol[r - 1], fidx[r] = fidx[r - 1];
                            fcol[r] = c, fidx[r] = x;
                        }
                        continue;
                    }
                    row.clear();
                    for (uint32_t q = a; q < z; q++) row.push_back({K(fcol[q]), {fcol[q], fidx[q]}});
                    std::sort(row.begin(), row.end(), [](auto &x, auto &y) { return x.first < y.first; });
                    for (size_t t = 0; t < row.size(); t++)
                        fcol[a + t] = row[t].second.first, fidx[a + t] = row[t].second.second;
                }
            });
    }
    clk.lap("layout: forward rows");
    // structure only (the device numeric phase fills the values): no host value arrays, the
    // device ones are zeroed in place
    std::vector<double> fval(vals ? nf : 0, 0.0);
    if (vals)
        parallel_for(nf, [&](int64_t lo, int64_t hi) {
            for (int64_t q = lo; q < hi; q++) fval[q] = f.Lx[fidx[q]];
        });
    // backward rows: L's columns (plus extra entries), keys descending; bidx[q] = CSC slot
    std::vector<uint32_t> bptr(N + 1, 0);
    for (int64_t j = 0; j < N; j++)
        bptr[j + 1] = bptr[j] + (uint32_t)(f.Lp[j + 1] - f.Lp[j]) + (uint32_t)(extra ? (*extra)[j].size() : 0);
    const bool bvals = vals || nextra > 0;
    std::vector<double> bval(bvals ? d.nnz : 0, 0.0);
    parallel_for(N, [&](int64_t lo, int64_t hi) {  // rows (columns of L) sort independently
        std::vector<std::pair<int64_t, std::pair<int32_t, int64_t>>> row;  // (key, (col, CSC slot | ~extra))
        for (int64_t j = lo; j < hi; j++) {
            const int64_t len = f.Lp[j + 1] - f.Lp[j];
            const uint32_t b = bptr[j];
            if ((!extra || (*extra)[j].empty()) && len <= kInsertionSortMax) {
                // short columns without extra entries: insertion sort (keys descending) in place
                int64_t src[kInsertionSortMax];
                for (int64_t t = 0; t < len; t++) {
                    const int64_t p = f.Lp[j] + t;
                    const int32_t c = f.Li[p];
                    const int64_t kc = K(c);
                    int64_t r = t;
                    for (; r > 0 && K(bcol[b + r - 1]) < kc; r--) bcol[b + r] = bcol[b + r - 1], src[r] = src[r - 1];
                    bcol[b + r] = c, src[r] = p;
                }
                for (int64_t t = 0; t < len; t++) {
                    if (vals) bval[b + t] = f.Lx[src[t]];
                    if (bsrc) bidx[b + t] = (int32_t)src[t];
                }
                continue;
            }
            row.clear();
            for (int64_t p = f.Lp[j]; p < f.Lp[j + 1]; p++) row.push_back({K(f.Li[p]), {f.Li[p], p}});
            if (extra)
                for (size_t t = 0; t < (*extra)[j].size(); t++) row.push_back({(*extra)[j][t].key, {(*extra)[j][t].col, ~(int64_t)t}});
            std::sort(row.begin(), row.end(), [](auto &x, auto &y) { return x.first > y.first; });
            for (size_t t = 0; t < row.size(); t++) {
                const int64_t src = row[t].second.second;
                bcol[b + t] = row[t].second.first;
                if (src < 0) bval[b + t] = (*extra)[j][~src].val;
                else if (vals) bval[b + t] = f.Lx[src];
                if (bsrc) bidx[b + t] = (int32_t)src;
            }
        }
    });
    clk.lap("layout: backward rows");
    if (fsrc) *fsrc = std::move(fidx);
    if (bsrc) *bsrc = std::move(bidx);
    // rounds whose blocks all fit the upper-round staging image (sptrsv_upper_kernel)
    d.round_fits.assign(s.round_ptr.empty() ? 0 : s.round_ptr.size() - 1, 1);
    for (size_t r = 0; r < d.round_fits.size(); r++)
        for (int64_t b = s.round_ptr[r]; b < s.round_ptr[r + 1]; b++) {
            const int64_t r0 = s.lvl_row[s.blk_lvl[b]], r1 = s.lvl_row[s.blk_lvl[b + 1]];
            if (r1 - r0 > d.sweep_rows[1] || fptr[r1] - fptr[r0] > (uint32_t)d.sweep_cap[1] ||
                bptr[r1] - bptr[r0] > (uint32_t)d.sweep_cap[1])
                d.round_fits[r] = 0;
        }
    // padding entries: clamped, unconditional loads may touch one entry past a block's end
    fcol.resize(fcol.size() + kFactorPadEntries, 0), bcol.resize(bcol.size() + kFactorPadEntries, 0);
    clk.lap("layout: round fits, padding");
    d.fptr.upload(fptr);
    d.fcol.upload(fcol);
    if (vals) {
        fval.resize(fval.size() + kFactorPadEntries, 0.0);
        d.fval.upload(fval);
    } else {
        d.fval.alloc((size_t)nf + kFactorPadEntries);
        CPK_HIP(hipMemset(d.fval.p, 0, d.fval.bytes()));
    }
    d.bptr.upload(bptr);
    d.bcol.upload(bcol);
    if (bvals) {
        bval.resize(bval.size() + kFactorPadEntries, 0.0);
        d.bval.upload(bval);
    } else {
        d.bval.alloc((size_t)d.nnz + kFactorPadEntries);
        CPK_HIP(hipMemset(d.bval.p, 0, d.bval.bytes()));
    }
    if (vals) d.D.upload(f.D);
    else d.D.alloc((size_t)N);
    d.perm.upload(f.perm);
    d.nblk = (int64_t)s.blk_row.size() - 1;
    d.nlvl = (int64_t)s.lvl_row.size() - 1;
    // the block records keep a level index and two flag bits in one int32 (kMetaL1Mask)
    if (d.nlvl > kMetaL1Mask) throw Error(CPK_ERR_UNSUPPORTED, "more sweep levels than the block records can index");
    std::vector<int32_t> bl(s.blk_lvl.begin(), s.blk_lvl.end()), lr(s.lvl_row.begin(), s.lvl_row.end());
    d.blk_lvl.upload(bl);
    d.lvl_row.upload(lr);
    d.round_ptr = s.round_ptr;
    // per-block metadata records for the pipelined round-0 kernel
    std::vector<int32_t> meta((size_t)d.nblk * 8);
    for (int64_t b = 0; b < d.nblk; b++) {
        const int64_t l0 = s.blk_lvl[b], l1 = s.blk_lvl[b + 1];
        const int64_t r0 = s.lvl_row[l0], r1 = s.lvl_row[l1];
        int32_t *m = &meta[(size_t)b * 8];
        m[0] = (int32_t)r0, m[1] = (int32_t)r1, m[2] = (int32_t)l0, m[3] = (int32_t)l1;
        m[4] = (int32_t)fptr[r0], m[5] = (int32_t)fptr[r1], m[6] = (int32_t)bptr[r0], m[7] = (int32_t)bptr[r1];
    }
    {
        const std::vector<int16_t> us = build_ufold(d, meta, s.round_ptr, fptr, fcol, bptr, bcol, [&](int64_t q) { return K(q); });
        mark_dataflow(meta, s.round_ptr, fptr, fcol, bptr, bcol, d.dataflow, d.colsweep, us, d.urow0, &d.hmodel);
    }
    d.meta.upload(meta);
    d.hmeta = meta;
    clk.lap("layout: uploads, block records, level-loop choice");
    d.round0_rows = -1;
    if (s.round_ptr.size() >= 2) {  // round 0 a leading, contiguous row range?
        int64_t r = 0;
        for (int64_t b = s.round_ptr[0]; b < s.round_ptr[1] && r >= 0; b++)
            r = meta[(size_t)b * 8] == r ? meta[(size_t)b * 8 + 1] : -1;
        d.round0_rows = r;
    }
    // round 0's forward entries as 16-bit block-local columns: a round-0 block holds whole
    // subtrees, so a row's forward columns (its descendants) are in its own block; checked here,
    // and the image is only built when it holds for every block
    d.fcol16.release();
    d.nnz16 = 0;
    if (s.round_ptr.size() >= 2 && !d.no_col16) {
        const int64_t b0 = s.round_ptr[0], nb0 = s.round_ptr[1] - b0;
        std::atomic<bool> bad{false};
        int64_t e_end = 0;
        for (int64_t b = b0; b < b0 + nb0; b++) e_end = std::max<int64_t>(e_end, meta[(size_t)b * 8 + 5]);
        parallel_for(nb0, [&](int64_t lo, int64_t hi) {  // blocks check independently
            for (int64_t b = b0 + lo; b < b0 + hi && !bad.load(std::memory_order_relaxed); b++) {
                const int32_t *m = &meta[(size_t)b * 8];
                bool ok = m[1] - m[0] <= INT16_MAX;
                for (int32_t e = m[4]; e < m[5] && ok; e++) ok = fcol[e] >= m[0] && fcol[e] < m[1];
                if (!ok) bad = true;
            }
        }, 1024);
        if (!bad) {
            std::vector<int16_t> c16((size_t)e_end + kFactorPadEntries, 0);
            parallel_for(nb0, [&](int64_t lo, int64_t hi) {
                for (int64_t b = b0 + lo; b < b0 + hi; b++) {
                    const int32_t *m = &meta[(size_t)b * 8];
                    for (int32_t e = m[4]; e < m[5]; e++) c16[e] = (int16_t)(fcol[e] - m[0]);
                }
            }, 1024);
            for (int64_t b = b0; b < b0 + nb0; b++) d.nnz16 += meta[(size_t)b * 8 + 5] - meta[(size_t)b * 8 + 4];
            d.fcol16.upload(c16);
        }
    }
    clk.lap("layout: int16 round-0 columns");
    build_chain(d, meta, fptr, fcol, bptr, bcol);
    clk.lap("layout: sweep chain");
}

// ---- SpMV launchers --------------------------------------------------------------------------
namespace {
struct EpiStore {
    double *y;
    const int *run;
    __device__ bool skip() const { return run && *run == 0; }
    __device__ const double *xvec(const double *x) const { return x; }
    __device__ double pre(int64_t) const { return 0.0; }
    __device__ void row(int64_t r, double acc, double) { y[r] = acc; }
    __device__ void finish() {}
};
struct EpiResid {
    const double *xin;
    int64_t neg_from;
    double *r;
    const int *run, *active;
    __device__ bool skip() const { return cpk::skip(run, active); }
    __device__ const double *xvec(const double *x) const { return x; }
    __device__ double pre(int64_t i) const { return xin[i]; }
    __device__ void row(int64_t i, double acc, double xi) {
        if (i >= neg_from) xi = -xi;
        r[i] = xi - acc;
    }
    __device__ void finish() {}
};
struct EpiResidSched {  // r(k) = xin(perm(k)) - (A y)(k), A and y in schedule order
    const double *xin;
    const int32_t *perm;  // null: xin is already the signed input in schedule order
    int64_t neg_from;
    double *r;
    const int *run;
    __device__ bool skip() const { return run && *run == 0; }
    __device__ const double *xvec(const double *x) const { return x; }
    __device__ double pre(int64_t i) const {
        if (!perm) return xin[i];
        const int32_t s = perm[i];
        const double x = xin[s];
        return s >= neg_from ? -x : x;
    }
    __device__ void row(int64_t i, double acc, double xi) { r[i] = xi - acc; }
    __device__ void finish() {}
};
template <class A = double>
struct EpiResidNorm {
    const double *xin;
    int64_t neg_from;
    double *r;
    double tol;
    int *active_out;
    RedBuf rb;
    const int *run, *active;
    A rr{}, xx{};
    static constexpr int kWaves = std::is_same<A, XAcc>::value ? 4 : CPK_SPMV_WAVES;
    __device__ bool skip() const { return cpk::skip(run, active); }
    __device__ const double *xvec(const double *x) {
        acc_init(rr, rb.xsub, 0, 2), acc_init(xx, rb.xsub, 1, 2);
        return x;
    }
    __device__ double pre(int64_t i) const { return xin[i]; }
    __device__ void row(int64_t i, double acc, double xi) {
        if (i >= neg_from) xi = -xi;
        double ri = xi - acc;
        r[i] = ri;
        dadd(rr, ri, ri);
        dadd(xx, xi, xi);
    }
    __device__ void finish() {
        A v[2] = {rr, xx};
        double tot[2];
        if (grid_sum<2>(v, rb, tot) && threadIdx.x == 0) {
            // while nit < nitref & (rNorm >= itref_tol * xNorm | force_itref)   (opLDL2.m:183)
            double rNorm = sqrt(tot[0]), xNorm = sqrt(tot[1]);
            *active_out = (rNorm >= tol * xNorm) ? 1 : 0;
        }
    }
};
}  // namespace

static inline int grid_of(const DMat &A) { return (int)A.nblk; }

template <class Epi>
static void spmv_launch(Ctx &c, const DMat &A, const double *x, int64_t col_min, const Epi &e) {
    const unsigned grid = A.ghosts() ? spmv_grid<Epi, true>(A.nblk) : spmv_grid<Epi, false>(A.nblk);
    if (A.ghosts())
        hipLaunchKernelGGL((spmv_stream<Epi, true>), dim3(grid), dim3(kBlock), 0, c.stream, A.ptr.p, A.col.p,
                           A.val.p, A.blk.p, A.nblk, x, col_min, e, (const double *)A.rbuf.p, A.nloc);
    else
        hipLaunchKernelGGL((spmv_stream<Epi, false>), dim3(grid), dim3(kBlock), 0, c.stream, A.ptr.p, A.col.p,
                           A.val.p, A.blk.p, A.nblk, x, col_min, e, (const double *)nullptr, (int64_t)0);
    CPK_HIP(hipGetLastError());
}

// ---- distributed halo ----------------------------------------------------
__global__ void gather_kernel(const double *__restrict__ x, const int32_t *__restrict__ idx, int64_t n,
                              double *__restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = x[idx[i]];
}

void launch_gather(Ctx &c, const double *x, const int32_t *idx, int64_t n, double *out) {
    if (n <= 0) return;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(256), 0, c.stream, x, idx, n, out);
    CPK_HIP(hipGetLastError());
}

void launch_halo(Ctx &c, const DMat &A, const double *x, bool packed) {
    if (!A.halo() || A.kmax == 0) return;
    if (!packed) launch_gather(c, x, A.send.p, A.nsend, A.sbuf.p);
    c.comm->allgather(A.sbuf.p, A.rbuf.p, (size_t)A.kstride, c.stream);
}

void make_dist_dmat(const DistCsr &a, int nranks, DMat &d) {
    make_dmat(a.a, d);
    d.nloc = a.nloc, d.kmax = a.kmax, d.kstride = a.kstride, d.nsend = (int64_t)a.send.size();
    d.send.upload(a.send);
    d.sbuf.alloc((size_t)std::max<int64_t>(a.kstride, 1));
    d.rbuf.alloc((size_t)std::max<int64_t>(a.kstride * nranks, 1));
    CPK_HIP(hipMemset(d.sbuf.p, 0, d.sbuf.bytes()));
    CPK_HIP(hipMemset(d.rbuf.p, 0, d.rbuf.bytes()));
}

__global__ void sum_slots_kernel(const double *__restrict__ slots, int P, int64_t n, double *__restrict__ out) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        double s = slots[j];
        for (int q = 1; q < P; q++) s += slots[(int64_t)q * n + j];
        out[j] = s;
    }
}
void launch_sum_slots(hipStream_t st, const double *slots, int P, size_t n, double *out) {
    if (!n) return;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(sum_slots_kernel, dim3(grid), dim3(256), 0, st, slots, P, (int64_t)n, out);
    CPK_HIP(hipGetLastError());
}

__global__ void sum_slots_i64_kernel(const int64_t *__restrict__ slots, int P, int64_t n, int64_t *__restrict__ out) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        int64_t s = slots[j];
        for (int q = 1; q < P; q++) s += slots[(int64_t)q * n + j];
        out[j] = s;
    }
}
void launch_sum_slots_i64(hipStream_t st, const int64_t *slots, int P, size_t n, int64_t *out) {
    if (!n) return;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(sum_slots_i64_kernel, dim3(grid), dim3(256), 0, st, slots, P, (int64_t)n, out);
    CPK_HIP(hipGetLastError());
}

void launch_spmv(Ctx &c, const DMat &A, const double *x, double *y, const int *run) {
    launch_halo(c, A, x);
    if (!A.nblk) return;
    spmv_launch(c, A, x, 0, EpiStore{y, run});
}

void launch_spmv_colmask(Ctx &c, const DMat &A, int64_t col_min, const double *x, double *y, const int *run) {
    launch_halo(c, A, x);
    if (!A.nblk) return;
    spmv_launch(c, A, x, col_min, EpiStore{y, run});
}

void launch_spmv_resid(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                       const int *run, const int *active, bool halo_packed) {
    launch_halo(c, A, y, halo_packed);
    if (!A.nblk) return;
    spmv_launch(c, A, y, 0, EpiResid{xin, neg_from, r, run, active});
}

void launch_spmv_resid_loc(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                           const int *run, const double *halo) {
    if (!A.nblk) return;
    const EpiResid e{xin, neg_from, r, run, nullptr};
    const unsigned grid = spmv_grid<EpiResid, true>(A.nblk);
    hipLaunchKernelGGL((spmv_stream<EpiResid, true>), dim3(grid), dim3(kBlock), 0, c.stream, A.ptr.p, A.col.p,
                       A.val.p, A.blk.p, A.nblk, y, (int64_t)0, e, halo, A.nloc);
    CPK_HIP(hipGetLastError());
}

void launch_spmv_resid_sched(Ctx &c, const DMat &A, const int32_t *perm, const double *xin, int64_t neg_from,
                             const double *y, double *r, const int *run) {
    if (!A.nblk) return;
    spmv_launch(c, A, y, 0, EpiResidSched{xin, perm, neg_from, r, run});
}

// the refinement predicate from the allreduced (|r|^2, |x|^2) (distributed mode)
__global__ void resid_norm_fin_kernel(const double *tot, double tol, int *active_out, const int *run,
                                      const int *active) {
    if (threadIdx.x || blockIdx.x || skip(run, active)) return;
    *active_out = (sqrt(tot[0]) >= tol * sqrt(tot[1])) ? 1 : 0;
}

void launch_spmv_resid_norm(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                            double tol, int *active_out, const int *run, const int *active, bool halo_packed) {
    launch_halo(c, A, y, halo_packed);
    const bool dist = c.dist();
    if (A.nblk) {
        c.ensure_partials((size_t)A.nblk * 2);
        const RedBuf rb = red_buf(c);
        if (c.exact())
            spmv_launch(c, A, y, 0, EpiResidNorm<XAcc>{xin, neg_from, r, tol, active_out, rb, run, active});
        else
            spmv_launch(c, A, y, 0, EpiResidNorm<>{xin, neg_from, r, tol, active_out, rb, run, active});
    } else if (dist) {  // no rows here: zero local sums
        c.ensure_partials(1);  // (and the exact digits, if exact_dots was switched on after the buffers were sized)
        if (c.exact()) CPK_HIP(hipMemsetAsync(c.xred.p, 0, 2 * kXW * sizeof(int64_t), c.stream));
        else CPK_HIP(hipMemsetAsync(c.red.p, 0, 2 * sizeof(double), c.stream));
    }
    if (dist) {
        allreduce_red(c, 2);
        hipLaunchKernelGGL(resid_norm_fin_kernel, dim3(1), dim3(64), 0, c.stream, (const double *)c.red.p, tol,
                           active_out, run, active);
        CPK_HIP(hipGetLastError());
    }
}

// ---- separator solve of the distributed apply ----------------------------
// Every rank solves the (replicated) separator rows T redundantly: forward from the allgathered
// payload (subtree values of every rank + the T inputs published by rank 0), then backward, each
// row subtracting its terms in the exported factor's order, exactly as the single-GPU sweep does.
// The results go to wT = w[nsub + t] (read by the local backward sweep as outside-block values)
// and, on rank 0, to the T dofs of y.  Two paths: the stepped solve of one workgroup below
// (T fits its LDS and step table), and the T sweep (dsep_sweep_setup) for any other T.
// Stepped separator solve, restructured for latency.  A one-pass kernel (r01-r03) walked each
// term with two dependent global loads; at S10 / 8 ranks T has 593 rows, 13 levels and rows of up
// to 49 payload terms, and it took ~160 us.  Here:
//  (1) tprefix_kernel, one wave per row across the chip: each forward row subtracts its LEADING
//      payload terms (coalesced loads, one gather, the subtractions in order on one lane) into
//      pre[t], and the payload terms of the rest of the row are pre-multiplied into their
//      records (read later against the 1.0 slot wt[nT]);
//  (2) tsolve_steps_kernel, one workgroup, stages the records in LDS and runs the levels as a
//      list of steps built at setup.  A step hands each lane of its first W waves one record
//      (value, meta).  A row chunk is a lead lane (row, length, flags) followed by its terms on
//      the next lanes of the same wave; each lane forms its product, and the lead subtracts the
//      chunk's products in the row's order.  No index is looked up at run time: a step costs
//      one record read, one gather, the chain, one store and, at the end of a level, a barrier.
//      The forward chains (up to 31 dependent subtractions per row, in the factor's order)
//      bound it: VALU issue, with up to four waves per SIMD in the wide levels.
// Row sums keep the exported factor's order: bit-identical.
constexpr int kTsolveThreads = 1024;
constexpr size_t kTsolveMaxLds = 160 * 1024;  // gfx950: 160 KB of LDS per workgroup
constexpr int kTsChunk = 32;                  // terms per row chunk
constexpr int kTsMaxSteps = 256;              // the step table lives in 4 VGPRs per lane
constexpr int64_t kTsMaxRows = 1 << 16;
// meta: a term lane holds its LDS column; a lead lane kTsLead | row | (length - 1) << 16 | flags
constexpr uint32_t kTsLead = 1u << 31, kTsFirst = 1u << 30, kTsLast = 1u << 29;
constexpr uint32_t kTsBarrier = 1u << 16;  // step table: waves | barrier after the step

// the T rows' Kp rows for the refinement residual (Precond::tkr); ptr null: none
struct TkrArgs {
    const int32_t *ptr = nullptr, *col = nullptr;
    const double *val = nullptr, *wT = nullptr;
};

// x of lane i + 1 (wave shift; the last lane gets 0)
__device__ __forceinline__ double ts_next_lane(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x130, 0xf, 0xf, true);  // wave_shl:1
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x130, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

// TKR (Precond::tkr, the refinement solve): the row's input is the T row's refinement residual
// xs_t - Kp row t * y, formed here first (the wave's products, added in Kp's column order from
// 0.0 by lane 0 through the same lane shifts): tkr_resid_kernel's arithmetic without its launch
__global__ __launch_bounds__(256) void tprefix_kernel(
    int nT, const int32_t *__restrict__ tk_ptr, const int32_t *__restrict__ tk_col, const double *__restrict__ tk_val,
    const int32_t *__restrict__ tr_ptr, const int32_t *__restrict__ tr_col, const double *__restrict__ tr_val,
    const int32_t *__restrict__ tr_slot, const int32_t *__restrict__ tf_src, const double *__restrict__ rbuf,
    double *__restrict__ pre, double *__restrict__ rec_v, const int *run, const int *active, TkrArgs tkr) {
    if (skip(run, active)) return;
    const int wv = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int t = blockIdx.x * 4 + wv;
    if (t >= nT) return;  // whole waves: the shifts below need every lane
    double acc = rbuf[tf_src[t]];
    if (tkr.ptr) {
        double sum = 0.0;
        const int q1 = tkr.ptr[t + 1];
        for (int e = tkr.ptr[t]; e < q1; e += kWave) {
            const int q = e + lane;
            double x = 0.0;
            if (q < q1) {
                const int32_t cq = tkr.col[q];
                x = tkr.val[q] * (cq < 0 ? tkr.wT[-cq - 1] : rbuf[cq]);
            }
            const int n = min(kWave, q1 - e);
            sum += x;
            for (int u = 1; u < n; u++) {
                x = ts_next_lane(x);
                sum += x;
            }
        }
        acc = acc - sum;
    }
    const int k1 = tk_ptr[t + 1];
    for (int e = tk_ptr[t]; e < k1; e += kWave) {
        const int q = e + lane;
        double x = q < k1 ? tk_val[q] * rbuf[tk_col[q]] : 0.0;
        // lane 0 subtracts the wave's products in order, shifted to it one lane at a time
        const int n = min(kWave, k1 - e);
        acc -= x;
        for (int u = 1; u < n; u++) {
            x = ts_next_lane(x);
            acc -= x;
        }
    }
    if (lane == 0) pre[t] = acc;
    for (int q = tr_ptr[t] + lane; q < tr_ptr[t + 1]; q += kWave) rec_v[tr_slot[q]] = tr_val[q] * rbuf[tr_col[q]];
}


// steps [s0, s1); woff: the first record of step s0 (in waves) on entry, of step s1 on exit
__device__ __forceinline__ void ts_steps(int s0, int s1, const int (&tab)[kTsMaxSteps / kWave], int &woff,
                                         const double *rv, const uint32_t *rm, double *wt, double &acc) {
    const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
    for (int s = s0; s < s1; s++) {
        int e = 0;
#pragma unroll
        for (int i = 0; i < kTsMaxSteps / kWave; i++)
            if ((s >> 6) == i) e = __builtin_amdgcn_readlane(tab[i], s & 63);
        const int W = e & 0xffff;
        if (wave < W) {  // whole waves: the shifts below need every lane
            const int r = (woff + wave) * kWave + lane;
            const double v = rv[r];
            const uint32_t m = rm[r];
            const bool lead = m & kTsLead;
            const double g = wt[m & 0xffffu];  // a term's column, or the lead's own row
            double x = lead ? 0.0 : v * g;
            if (lead && (m & kTsFirst)) acc = g;
            // each lead subtracts the products of the next nw lanes in order, shifted to it one
            // lane at a time (no LDS traffic).  Lane 0 leads the wave's first chunk, and every
            // chunk of a wave is padded to the same length nw, so no lane needs a select.
            const int nw = (int)((__builtin_amdgcn_readfirstlane(m) >> 16) & 31u) + 1;
            for (int k = 0; k < nw; k++) {
                x = ts_next_lane(x);
                acc -= x;
            }
            if (lead && (m & kTsLast)) wt[m & 0xffffu] = acc;
        }
        woff += W;
        if (e & kTsBarrier) __syncthreads();
    }
}

// GREC: the records stay in HBM (a separator whose records do not fit in LDS); each step then
// waits for its record loads, which is still several times faster than the one-pass kernel
template <bool GREC>
__global__ __launch_bounds__(kTsolveThreads) void tsolve_steps_kernel(
    int nT, int nsf, int nsb, int nrec, const double *__restrict__ rec_v, const uint32_t *__restrict__ rec_m,
    const int32_t *__restrict__ steps, const double *__restrict__ pre, const double *__restrict__ DT,
    const int32_t *__restrict__ tdof, int ntdof, double *wT, double *y, int add, const int *run, const int *active,
    const int32_t *__restrict__ hslot, double *hbuf) {
    // LDS: wt[nT + 1, even] | rv[nrec] | rm[nrec] (the records: staged unless GREC)
    extern __shared__ __attribute__((aligned(16))) double tsw[];
    if (skip(run, active)) return;
    const int tid = threadIdx.x, lane = tid % kWave;
    double *wt = tsw;
    const double *rv = GREC ? rec_v : wt + ((nT + 2) & ~1);
    const uint32_t *rm = GREC ? rec_m : reinterpret_cast<const uint32_t *>(rv + nrec);
    int tab[kTsMaxSteps / kWave];  // lane i of tab[k]: step 64k + i (waves | barrier)
#pragma unroll
    for (int k = 0; k < kTsMaxSteps / kWave; k++) {
        const int s = k * kWave + lane;
        tab[k] = s < nsf + nsb ? steps[s] : 0;
    }
    {  // stage: every load in flight at once
        constexpr int U = 8;
        for (int i0 = tid; i0 <= nT; i0 += kTsolveThreads) wt[i0] = pre[i0];  // pre[nT] = 1.0
        double *srv = wt + ((nT + 2) & ~1);
        uint32_t *srm = reinterpret_cast<uint32_t *>(srv + nrec);
        for (int i0 = tid; i0 < (GREC ? 0 : nrec); i0 += U * kTsolveThreads) {
            double a[U];
            uint32_t b[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int i = i0 + u * kTsolveThreads;
                a[u] = i < nrec ? rec_v[i] : 0.0;
                b[u] = i < nrec ? rec_m[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int i = i0 + u * kTsolveThreads;
                if (i < nrec) srv[i] = a[u], srm[i] = b[u];
            }
        }
    }
    __syncthreads();
    double acc = 0.0;
    int woff = 0;
    ts_steps(0, nsf, tab, woff, rv, rm, wt, acc);  // forward: the rest of each row
    // backward: every row's diagonal step first (D is diagonal, and a row's terms read only rows
    // of later levels, final by the time it runs), then the rows' terms
    for (int t = tid; t < nT; t += kTsolveThreads) wt[t] = wt[t] / DT[t];
    __syncthreads();
    ts_steps(nsf, nsf + nsb, tab, woff, rv, rm, wt, acc);
    for (int t = tid; t < nT; t += kTsolveThreads) {
        wT[t] = wt[t];
        if (t < ntdof) {
            const int32_t d = tdof[t];
            const double o = add ? y[d] + wt[t] : wt[t];
            y[d] = o;
            if (hslot && hslot[d] >= 0) hbuf[hslot[d]] = o;  // the Kp halo of y (PackArgs)
        }
    }
}

namespace {
// Packs one direction's level rows into steps: a step has kTsolveThreads lanes in waves of 64,
// a row chunk takes a lead lane plus one lane per term inside one wave.  Records are stored by
// step, for the step's used waves only.
struct StepPacker {
    static constexpr int kWaves = kTsolveThreads / kWave;
    struct Lane {
        double v = 0.0;
        uint32_t m = 0;
        int64_t term = -1;  // caller's term id (slot callback), -1: none
    };
    std::vector<std::vector<Lane>> steps;  // kTsolveThreads lanes each
    std::vector<int> used_waves;           // 1 + the last wave holding a chunk
    std::vector<bool> barrier;
    uint32_t one_col = 0;                  // LDS column of the 1.0 slot (nT)
    // terms(t): (value, LDS column, term id) of row t in order
    template <class Terms>
    void level(const std::vector<int32_t> &rows, Terms terms) {
        if (rows.empty()) return;
        const size_t first = steps.size();
        std::vector<std::array<int, kWaves>> used;
        auto ensure = [&](size_t k) {
            while (used.size() <= k) {
                used.push_back({});
                steps.emplace_back(kTsolveThreads);
                used_waves.push_back(0);
                barrier.push_back(false);
            }
        };
        // a chunk of n terms padded to npad (the wave's chunk length): pad lanes hold 0.0
        // against the 1.0 slot, so subtracting their products leaves the sum unchanged
        auto put = [&](int32_t t, size_t k, int w, int lane0, const std::vector<std::tuple<double, int32_t, int64_t>> &tv,
                       size_t j0, size_t n, bool fst, bool lst, size_t npad) {
            auto &st = steps[first + k];
            Lane &ld = st[(size_t)(w * kWave + lane0)];
            ld.m = kTsLead | (uint32_t)t | ((uint32_t)(npad - 1) << 16) | (fst ? kTsFirst : 0u) | (lst ? kTsLast : 0u);
            for (size_t j = 0; j < npad; j++) {
                Lane &l = st[(size_t)(w * kWave + lane0 + 1) + j];
                if (j < n)
                    l.v = std::get<0>(tv[j0 + j]), l.m = (uint32_t)std::get<1>(tv[j0 + j]), l.term = std::get<2>(tv[j0 + j]);
                else
                    l.v = 0.0, l.m = one_col;
            }
            used_waves[first + k] = std::max(used_waves[first + k], w + 1);
        };
        std::vector<std::pair<size_t, int32_t>> single;
        for (int32_t t : rows) {
            const auto tv = terms(t);
            const size_t n = tv.size();
            if (n <= (size_t)kTsChunk) {
                single.push_back({n, t});
                continue;
            }
            const size_t k = (n + kTsChunk - 1) / kTsChunk;  // a wave of its own in k consecutive steps
            for (size_t s = 0;; s++) {
                ensure(s + k - 1);
                int w = 0;
                for (; w < kWaves; w++) {
                    bool fr = true;
                    for (size_t j = 0; j < k && fr; j++) fr = used[s + j][w] == 0;
                    if (fr) break;
                }
                if (w == kWaves) continue;
                for (size_t j = 0; j < k; j++) {
                    used[s + j][w] = kWave;
                    const size_t nj = std::min<size_t>(kTsChunk, n - j * kTsChunk);
                    put(t, s + j, w, 0, tv, j * kTsChunk, nj, j == 0, j == k - 1, nj);
                }
                break;
            }
        }
        // the other rows longest first, a wave at a time: every chunk of a wave is padded to the
        // wave's first (longest) one, so the wave's chain length is uniform (kernel: no selects)
        std::stable_sort(single.begin(), single.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
        size_t i = 0;
        for (size_t s = 0; i < single.size(); s++) {
            ensure(s);
            for (int w = 0; w < kWaves && i < single.size(); w++) {
                if (used[s][w]) continue;
                const size_t L = single[i].first;
                int lane = 0;
                while (i < single.size() && lane + (int)L + 1 <= kWave) {
                    const int32_t t = single[i].second;
                    put(t, s, w, lane, terms(t), 0, single[i].first, true, true, L);
                    lane += (int)L + 1;
                    i++;
                }
                used[s][w] = kWave;
            }
        }
        barrier.back() = true;
    }
};
}  // namespace

void dsep_stage(DSep &T, const RankPlan &rp) {
    const int64_t nT = T.nT;
    T.lds = 0;
    if (nT <= 0 || nT >= kTsMaxRows) return;
    // forward rows: leading payload terms (tprefix_kernel) | the rest, from the first T term on
    std::vector<int32_t> kp(nT + 1, 0), kc, rptr(nT + 1, 0), rcol, rslot;
    std::vector<double> kv, rval;
    std::vector<int64_t> rest0(nT);
    for (int64_t t = 0; t < nT; t++) {
        int64_t e = rp.tf_ptr[t];
        for (; e < rp.tf_ptr[t + 1] && rp.tf_col[e] >= 0; e++) kc.push_back(rp.tf_col[e]), kv.push_back(rp.tf_val[e]);
        kp[t + 1] = (int32_t)kc.size();
        rest0[t] = e;
    }
    StepPacker P;
    P.one_col = (uint32_t)nT;
    using TV = std::vector<std::tuple<double, int32_t, int64_t>>;
    auto rows_of = [&](int64_t l, bool bwd) {
        std::vector<int32_t> r;
        for (int64_t q = rp.tlev_ptr[l]; q < rp.tlev_ptr[l + 1]; q++) {
            const int32_t t = rp.tlev_rows[q];
            if (bwd ? rp.tb_ptr[t + 1] > rp.tb_ptr[t] : rp.tf_ptr[t + 1] > rest0[t]) r.push_back(t);
        }
        return r;
    };
    // forward terms: T rows against wt, payload terms (pre-multiplied per solve) against wt[nT]
    for (int64_t l = 0; l < T.nlev; l++)
        P.level(rows_of(l, false), [&](int32_t t) {
            TV tv;
            for (int64_t e = rest0[t]; e < rp.tf_ptr[t + 1]; e++)
                tv.emplace_back(rp.tf_col[e] >= 0 ? 0.0 : rp.tf_val[e],
                                rp.tf_col[e] >= 0 ? (int32_t)nT : (int32_t)(-rp.tf_col[e] - 1),
                                rp.tf_col[e] >= 0 ? e : (int64_t)-1);
            return tv;
        });
    T.nsf = (int64_t)P.steps.size();
    for (int64_t l = T.nlev - 1; l >= 0; l--)
        P.level(rows_of(l, true), [&](int32_t t) {
            TV tv;
            for (int64_t e = rp.tb_ptr[t]; e < rp.tb_ptr[t + 1]; e++) tv.emplace_back(rp.tb_val[e], rp.tb_col[e], (int64_t)-1);
            return tv;
        });
    T.nsb = (int64_t)P.steps.size() - T.nsf;
    if (T.nsf + T.nsb > kTsMaxSteps) return;
    // records of the used waves, step by step
    std::vector<double> rv;
    std::vector<uint32_t> rm;
    std::vector<int32_t> tab;
    std::vector<int64_t> pay_slot(rp.tf_col.size(), -1);
    for (size_t s = 0; s < P.steps.size(); s++) {
        tab.push_back(P.used_waves[s] | (P.barrier[s] ? (int32_t)kTsBarrier : 0));
        for (int i = 0; i < P.used_waves[s] * kWave; i++) {
            const auto &l = P.steps[s][(size_t)i];
            if (l.term >= 0) pay_slot[(size_t)l.term] = (int64_t)rv.size();
            rv.push_back(l.v), rm.push_back(l.m);
        }
    }
    for (int64_t t = 0; t < nT; t++) {
        for (int64_t e = rest0[t]; e < rp.tf_ptr[t + 1]; e++)
            if (rp.tf_col[e] >= 0) rcol.push_back(rp.tf_col[e]), rval.push_back(rp.tf_val[e]), rslot.push_back((int32_t)pay_slot[(size_t)e]);
        rptr[t + 1] = (int32_t)rcol.size();
    }
    T.tk_ptr.upload(kp), T.tk_col.upload(kc), T.tk_val.upload(kv);
    T.tr_ptr.upload(rptr), T.tr_col.upload(rcol), T.tr_val.upload(rval), T.tr_slot.upload(rslot);
    T.rec_v.upload(rv), T.rec_m.upload(rm), T.steps.upload(tab);
    T.nrec = (int64_t)rv.size();
    std::vector<double> pre(nT + 1, 0.0);
    pre[nT] = 1.0;
    T.pre.upload(pre);
    const size_t lds = 8 * (size_t)((nT + 2) & ~1) + 12 * (size_t)T.nrec;
    T.lds = lds <= kTsolveMaxLds ? lds : 0;
    T.lds_g = 8 * (size_t)((nT + 2) & ~1) <= kTsolveMaxLds ? 8 * (size_t)((nT + 2) & ~1) : 0;
}

// The T sweep.  T's rows are a factor of their own: L_T's columns are the backward rows tb_*
// (the rows below t, in T's pivot order), so its elimination tree is parent(t) = min tb_col,
// and build_schedule cuts it into blocks and rounds like a rank's subtrees, with each row's
// payload terms as extra forward entries.  The layout is a DFactor over the combined vector
// rbuf = [payload of every rank (P * kt); T rows in schedule order]: a forward entry on payload
// position p reads rbuf[p] (outside every block: pre-multiplied at staging, as any reference to
// an earlier round), one on T row t' reads rbuf[base + q(t')], a T row's input is rbuf[tf_src[t]]
// (perm), and the backward rows read the T region only.  Each row keeps tf_* / tb_* order -- the
// exported factor's -- so the block kernels give the stepped solve's bits; nothing limits T's
// size or its number of levels.
void dsep_sweep_setup(Ctx &c, DSep &T, const RankPlan &rp, int P) {
    const int64_t nT = T.nT, base = (int64_t)P * T.kt, NT = base + nT;
    T.tsweep = false;
    if (nT <= 0) return;
    if (NT > (int64_t)INT32_MAX / 2) throw Error(CPK_ERR_UNSUPPORTED, "separator payload too large");
    // L_T (CSC: column t holds the rows below it) and the etree
    Factor f;
    f.N = nT;
    f.Lp.assign((size_t)nT + 1, 0);
    f.parent.assign((size_t)nT, -1);
    std::vector<int64_t> xf((size_t)nT, 0);
    for (int64_t t = 0; t < nT; t++) {
        for (int64_t e = rp.tb_ptr[t]; e < rp.tb_ptr[t + 1]; e++) {
            const int32_t i = rp.tb_col[e];
            f.Li.push_back(i);
            if (f.parent[t] < 0 || i < f.parent[t]) f.parent[t] = i;
        }
        f.Lp[t + 1] = (int64_t)f.Li.size();
        for (int64_t e = rp.tf_ptr[t]; e < rp.tf_ptr[t + 1]; e++) xf[t] += rp.tf_col[e] >= 0;
    }
    const SweepConfig sw = dist_sweep_default();
    Schedule S = build_schedule(f, sw.rows[0], sw.cap[0], sw.rows[1], sw.cap[1], sw.sub0, nullptr, &xf);
    std::vector<int32_t> q((size_t)nT);
    for (int64_t k = 0; k < nT; k++) q[S.order[k]] = (int32_t)k;
    DFactor &d = T.tsw;
    for (int i = 0; i < 2; i++) d.sweep_rows[i] = sw.rows[i], d.sweep_cap[i] = sw.cap[i], d.sweep_threads[i] = sw.threads[i];
    d.pipelined = true, d.no_upper = false, d.no_col16 = true, d.fuse_last = false, d.skip0 = false;
    d.dataflow = c.opts.no_dataflow ? 1 : (c.opts.all_dataflow ? 2 : 0);
    d.colsweep = c.opts.no_colsweep ? 1 : (c.opts.all_colsweep ? 2 : 0);
    d.N = NT;
    std::vector<uint32_t> fptr((size_t)NT + 1, 0), bptr((size_t)NT + 1, 0);
    std::vector<int32_t> fcol, bcol, perm((size_t)NT, 0);
    std::vector<double> fval, bval, D((size_t)NT, 0.0);  // payload rows: never solved
    for (int64_t k = 0; k < nT; k++) {  // rows in schedule order
        const int32_t t = S.order[k];
        for (int64_t e = rp.tf_ptr[t]; e < rp.tf_ptr[t + 1]; e++) {
            const int32_t cc = rp.tf_col[e];
            fcol.push_back(cc >= 0 ? cc : (int32_t)(base + q[(size_t)(-cc - 1)]));
            fval.push_back(rp.tf_val[e]);
        }
        for (int64_t e = rp.tb_ptr[t]; e < rp.tb_ptr[t + 1]; e++) {
            bcol.push_back((int32_t)(base + q[(size_t)rp.tb_col[e]]));
            bval.push_back(rp.tb_val[e]);
        }
        fptr[base + k + 1] = (uint32_t)fcol.size();
        bptr[base + k + 1] = (uint32_t)bcol.size();
        perm[base + k] = rp.tf_src[t];
        D[base + k] = rp.DT[t];
    }
    for (int64_t r = 0; r < base; r++) fptr[r + 1] = 0, bptr[r + 1] = 0;  // payload rows: no entries
    d.nnz = (int64_t)fcol.size();
    fcol.resize(fcol.size() + kFactorPadEntries, 0), bcol.resize(bcol.size() + kFactorPadEntries, (int32_t)base);
    fval.resize(fval.size() + kFactorPadEntries, 0.0), bval.resize(bval.size() + kFactorPadEntries, 0.0);
    d.nblk = (int64_t)S.blk_row.size() - 1;
    d.nlvl = (int64_t)S.lvl_row.size() - 1;
    if (d.nlvl > kMetaL1Mask) throw Error(CPK_ERR_UNSUPPORTED, "more sweep levels than the block records can index");
    std::vector<int32_t> bl(S.blk_lvl.begin(), S.blk_lvl.end()), lr(S.lvl_row.size());
    for (size_t i = 0; i < lr.size(); i++) lr[i] = (int32_t)(base + S.lvl_row[i]);
    std::vector<int32_t> meta((size_t)d.nblk * 8);
    d.round_fits.assign(S.round_ptr.size() - 1, 1);
    for (int64_t b = 0; b < d.nblk; b++) {
        const int64_t r0 = base + S.lvl_row[S.blk_lvl[b]], r1 = base + S.lvl_row[S.blk_lvl[b + 1]];
        int32_t *m = &meta[(size_t)b * 8];
        m[0] = (int32_t)r0, m[1] = (int32_t)r1, m[2] = (int32_t)S.blk_lvl[b], m[3] = (int32_t)S.blk_lvl[b + 1];
        m[4] = (int32_t)fptr[r0], m[5] = (int32_t)fptr[r1], m[6] = (int32_t)bptr[r0], m[7] = (int32_t)bptr[r1];
    }
    {
        // row base + k is T row S.order[k]: its entries are in T's order (mark_dataflow checks it)
        const std::vector<int16_t> us = build_ufold(d, meta, S.round_ptr, fptr, fcol, bptr, bcol,
                    [&](int64_t q) { return q < base ? q - base : (int64_t)S.order[(size_t)(q - base)]; });
        mark_dataflow(meta, S.round_ptr, fptr, fcol, bptr, bcol, d.dataflow, d.colsweep, us, d.urow0, nullptr);
    }
    for (size_t r = 0; r < d.round_fits.size(); r++)
        for (int64_t b = S.round_ptr[r]; b < S.round_ptr[r + 1]; b++) {
            const int32_t *m = &meta[(size_t)b * 8];
            if (m[1] - m[0] > d.sweep_rows[1] || m[5] - m[4] > d.sweep_cap[1] || m[7] - m[6] > d.sweep_cap[1])
                d.round_fits[r] = 0;
        }
    d.fptr.upload(fptr), d.fcol.upload(fcol), d.fval.upload(fval);
    d.bptr.upload(bptr), d.bcol.upload(bcol), d.bval.upload(bval);
    d.D.upload(D), d.perm.upload(perm);
    d.blk_lvl.upload(bl), d.lvl_row.upload(lr), d.meta.upload(meta);
    d.hmeta = meta;
    d.round_ptr = S.round_ptr;
    d.round0_rows = -1;
    plan_round0(c, d, nullptr);
    // the T sweep's upper rounds as sweep chains (forward, backward): on the +-64 window at P = 8
    // T is 6128 rows in 8 rounds, 14 upper-round launches per T solve
    d.no_chain = c.opts.no_chain, d.chain_wide = c.opts.chain_wide;
    build_chain(d, meta, fptr, fcol, bptr, bcol);
    T.tsw_q.upload(q);
    T.tsw_base = base;
    T.tsweep = true;
}

// payload: w of this rank's rows that separator rows read, then (rank 0) the T inputs +-x[tdof]
// (and, with piggy, kSepPiggy values of a solver's into the spare slots [kt_data, kt))
__global__ void tpack_kernel(const double *__restrict__ w, const int32_t *__restrict__ send, int nsend,
                             const double *__restrict__ x, int64_t neg_from, const int32_t *__restrict__ tdof,
                             int ntdof, double *__restrict__ out, const double *__restrict__ piggy, int kt_data) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nsend) out[i] = w[send[i]];
    else if (i < nsend + ntdof) {
        const int32_t d = tdof[i - nsend];
        const double v = x[d];
        out[i] = d >= neg_from ? -v : v;
    }
    if (piggy && blockIdx.x == 0 && threadIdx.x < kSepPiggy) out[kt_data + threadIdx.x] = piggy[threadIdx.x];
}

void launch_sep_exchange(Ctx &c, const DSep &S, const double *w, const double *x, int64_t neg_from,
                         const double *piggy_src, bool packed) {
    if (S.kt == 0) return;
    const int64_t n = std::max<int64_t>(S.nsend + S.ntdof, piggy_src ? 1 : 0);
    if (n > 0 && !packed)
        hipLaunchKernelGGL(tpack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c.stream, w, S.send.p,
                           (int)S.nsend, x, neg_from, S.tdof.p, (int)S.ntdof, S.sbuf.p, piggy_src, (int)S.kt_data);
    CPK_HIP(hipGetLastError());
    c.comm->allgather(S.sbuf.p, S.rbuf.p, (size_t)S.kt, c.stream);
}

__global__ void tkr_resid_kernel(int nT, const int32_t *__restrict__ ptr, const int32_t *__restrict__ col,
                                 const double *__restrict__ val, const int32_t *__restrict__ tf_src,
                                 const double *__restrict__ wT, double *rbuf, const int *run, const int *active) {
    if (skip(run, active)) return;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nT) return;
    double acc = 0.0;  // the residual SpMV's row: products in Kp's column order, summed from 0.0
    for (int e = ptr[t]; e < ptr[t + 1]; e++) {
        const int32_t c = col[e];
        const double p = val[e] * (c < 0 ? wT[-c - 1] : rbuf[c]);
        acc += p;
    }
    rbuf[tf_src[t]] = rbuf[tf_src[t]] - acc;
}

void launch_tkr_resid(Ctx &c, const DSep &S, const int32_t *ptr, const int32_t *col, const double *val,
                      const double *wT, const int *run, const int *active) {
    if (S.nT == 0) return;
    hipLaunchKernelGGL(tkr_resid_kernel, dim3((unsigned)((S.nT + 255) / 256)), dim3(256), 0, c.stream, (int)S.nT, ptr,
                       col, val, S.tf_src.p, wT, S.rbuf.p, run, active);
    CPK_HIP(hipGetLastError());
}

// the T sweep's epilogue: wT in T order, rank 0's T dofs of y (and their Kp halo slots)
__global__ void tsep_out_kernel(int nT, const int32_t *__restrict__ q, const double *__restrict__ wsw,
                                const int32_t *__restrict__ tdof, int ntdof, double *wT, double *y, int add,
                                const int *run, const int *active, const int32_t *__restrict__ hslot, double *hbuf) {
    if (skip(run, active)) return;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nT; t += gridDim.x * blockDim.x) {
        const double v = wsw[q[t]];
        wT[t] = v;
        if (t < ntdof) {
            const int32_t d = tdof[t];
            const double o = add ? y[d] + v : v;
            y[d] = o;
            if (hslot && hslot[d] >= 0) hbuf[hslot[d]] = o;
        }
    }
}

// LDS of the stepped separator solve: up to 64 KB always, up to kTsolveMaxLds when the device
// grants the kernels that much dynamic LDS (asked once)
bool sep_lds_fits(size_t bytes) {
    static const bool lds_attr = [] {
        return hipFuncSetAttribute((const void *)tsolve_steps_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kTsolveMaxLds) == hipSuccess &&
               hipFuncSetAttribute((const void *)tsolve_steps_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kTsolveMaxLds) == hipSuccess;
    }();
    return bytes && (bytes <= 64 * 1024 || lds_attr);
}

// the stepped solve can run T: records staged in LDS, or (records in HBM: tsolve_global, or
// staged records too large) the rest of its image -- one predicate for setup (precond.cpp: else
// the T sweep is built) and launch (launch_sep_solve), so the two cannot disagree
bool sep_steps_fit(const DSep &S) {
    const bool grec = S.tsolve_global || !sep_lds_fits(S.lds);
    return S.nrec > 0 && sep_lds_fits(grec ? S.lds_g : S.lds);
}

void launch_sep_solve(Ctx &c, const DSep &S, double *wT, double *y, bool add, const int *run, const int *active,
                      const int32_t *hslot, double *hbuf, const int32_t *tkr_ptr, const int32_t *tkr_col,
                      const double *tkr_val, const double *tkr_yT) {
    if (!tkr_yT) tkr_yT = wT;
    if (S.nT == 0) return;
    const bool grec = S.tsolve_global || !sep_lds_fits(S.lds);  // engine option: records in HBM
    const size_t lds = grec ? S.lds_g : S.lds;
    const TkrArgs tkr{tkr_ptr, tkr_col, tkr_val, tkr_yT};  // y's T values (wT itself: this solve writes it last)
    if (!S.tsweep && sep_steps_fit(S)) {
        hipLaunchKernelGGL(tprefix_kernel, dim3((unsigned)((S.nT + 3) / 4)), dim3(256), 0, c.stream, (int)S.nT,
                           S.tk_ptr.p, S.tk_col.p, S.tk_val.p, S.tr_ptr.p, S.tr_col.p, S.tr_val.p, S.tr_slot.p,
                           S.tf_src.p, S.rbuf.p, S.pre.p, S.rec_v.p, run, active, tkr);
        if (grec)
            hipLaunchKernelGGL(tsolve_steps_kernel<true>, dim3(1), dim3(kTsolveThreads), lds, c.stream, (int)S.nT,
                               (int)S.nsf, (int)S.nsb, (int)S.nrec, (const double *)S.rec_v.p,
                               (const uint32_t *)S.rec_m.p, S.steps.p, (const double *)S.pre.p, (const double *)S.DT.p,
                               S.tdof.p, (int)S.ntdof, wT, y, add ? 1 : 0, run, active, hslot, hbuf);
        else
            hipLaunchKernelGGL(tsolve_steps_kernel<false>, dim3(1), dim3(kTsolveThreads), lds, c.stream, (int)S.nT,
                               (int)S.nsf, (int)S.nsb, (int)S.nrec, (const double *)S.rec_v.p,
                               (const uint32_t *)S.rec_m.p, S.steps.p, (const double *)S.pre.p, (const double *)S.DT.p,
                               S.tdof.p, (int)S.ntdof, wT, y, add ? 1 : 0, run, active, hslot, hbuf);
        CPK_HIP(hipGetLastError());
        return;
    }
    if (!S.tsweep) throw Error(CPK_ERR_UNSUPPORTED, "internal: separator solve without a path");
    // the T sweep: [payload; T] in rbuf; forward (input rbuf[tf_src[t]], the T rows' residual
    // formed first when tkr), backward, then wT and rank 0's T dofs
    if (tkr_ptr) launch_tkr_resid(c, S, tkr_ptr, tkr_col, tkr_val, tkr_yT, run, active);
    launch_sptrsv_fwd(c, S.tsw, S.rbuf.p, INT64_MAX, S.rbuf.p, run, active);
    launch_sptrsv_bwd(c, S.tsw, S.rbuf.p, nullptr, false, run, active);
    const int grid = (int)std::min<int64_t>((S.nT + 255) / 256, 1024);
    hipLaunchKernelGGL(tsep_out_kernel, dim3(grid), dim3(256), 0, c.stream, (int)S.nT, S.tsw_q.p,
                       (const double *)(S.rbuf.p + S.tsw_base), S.tdof.p, (int)S.ntdof, wT, y, add ? 1 : 0, run, active,
                       hslot, hbuf);
    CPK_HIP(hipGetLastError());
}

// ---- level-scheduled triangular sweeps -------------------------------------------------------
// One workgroup per schedule block.  A block holds whole elimination subtrees; its rows are
// contiguous and grouped by intra-block level, so a level is a contiguous row range and the
// only synchronisation inside a block is a workgroup barrier between levels.  Rows of other
// blocks that a block reads were finished by an earlier launch (earlier round).
//
// Staged path (the block fits in LDS): phase 1 streams the block's row pointers, entries and
// inputs from HBM with consecutive lanes on consecutive addresses, and folds every reference
// to a row OUTSIDE the block into its product val*w[col] right away (that value is final);
// phase 2 runs the levels entirely out of LDS; phase 3 writes the block's rows back
// contiguously.  Each row still subtracts its terms in the reference's order, one rounding per
// product and per subtraction, so the result is bit-identical to the direct path.
// LDS image of a staged block (dynamic shared memory, sized per launch):
//   double w[R + 1] | double v[CAP + 8] | int16 c[CAP + 8] | int16 p[R + 1] | int16 lv[R + 1] | int16 ps[R + 1]
constexpr int kSweepPad = 8;
#define CPK_UPPER_CH(bwd) ((bwd) ? CPK_UPPER_CH_BWD : CPK_UPPER_CH_FWD)
#ifndef CPK_PIPE_CH
#define CPK_PIPE_CH 2  // entries per LDS round trip in the round-0 level loop
#endif  // entry arrays padded for the branchless 8-entry chunks
struct SweepLds {
    double *w, *v;
    int16_t *c, *p, *lv, *ps;
    __device__ SweepLds(char *smem, int R, int CAP) {
        w = reinterpret_cast<double *>(smem);
        v = w + R + 1;  // w[R]: the 1.0 slot of sweep_levels<..., ONE>
        c = reinterpret_cast<int16_t *>(v + CAP + kSweepPad);
        p = c + CAP + kSweepPad;
        lv = p + R + 1;
        ps = lv + R + 1;
    }
};
__host__ __device__ constexpr size_t sweep_lds_bytes_dev(int R, int CAP) {
    return ((size_t)8 * (R + 1) + 10 * ((size_t)CAP + kSweepPad) + 6 * ((size_t)R + 1) + 15) & ~(size_t)15;
}
size_t sweep_lds_bytes(int R, int CAP) { return sweep_lds_bytes_dev(R, CAP); }

// Outside-block prefix: a row's leading terms that refer to rows finished by earlier launches
// are already products in LDS (c < 0).  Subtracting them here, every row at once, takes them
// off the level-by-level critical path; the level phase then continues each row from ps[k].
// Same operations in the same order, so the result is bit-identical.  This is what makes the
// upper rounds cheap: a separator row's many references into the subtrees below are all
// outside its block.
template <int TPB, int OUTC = -1>  // OUTC: column marking outside terms (-1, or R for the 1.0 slot)
__device__ __forceinline__ void fold_prefix(SweepLds &S, int nr, int tid = -1, int outc = OUTC) {
    if (tid < 0) tid = threadIdx.x;
    for (int i = tid; i < nr; i += TPB) {
        int e = S.p[i];
        const int e1 = S.p[i + 1];
        double acc = S.w[i];
        for (;;) {  // eight entries per LDS round trip; absent / stopped terms subtract +0.0
            int c[kSweepPad];
            double v[kSweepPad];
#pragma unroll
            for (int j = 0; j < kSweepPad; j++) c[j] = S.c[e + j], v[j] = S.v[e + j];
            int t = 0;
#pragma unroll
            for (int j = 0; j < kSweepPad; j++) {
                const bool take = t == j && e + j < e1 && (OUTC < 0 ? c[j] < 0 : c[j] == outc);
                acc -= take ? v[j] : 0.0;
                t += take;
            }
            e += t;
            if (t < kSweepPad) break;
        }
        S.w[i] = acc;
        S.ps[i] = (int16_t)e;
    }
    __syncthreads();
}

// fold_prefix with the prefix lengths known (UFold, counted at layout): ps[k] is set by the
// staging, so the fold is a plain run of subtractions of staged products -- 16 per pass, loads
// first -- with no per-term column test.  fold_prefix spends ~12 instructions per term on the
// test and its select chain (~140 cycles per term on the ±64 window's separator rows of ~190
// leading outside terms, r05 stamps); here a term is a load and a subtraction.  Same terms, same
// order: bit-identical.
template <int TPB>
__device__ __forceinline__ void fold_known(SweepLds &S, int nr, int tid) {
    constexpr int K = 16;
    for (int i = tid; i < nr; i += TPB) {
        int e = S.p[i];
        const int e1 = S.ps[i];
        double acc = S.w[i];
        for (; e + K <= e1; e += K) {
            double v[K];
#pragma unroll
            for (int j = 0; j < K; j++) v[j] = S.v[e + j];
#pragma unroll
            for (int j = 0; j < K; j++) acc -= v[j];
        }
        for (; e < e1; e++) acc -= S.v[e];
        S.w[i] = acc;
    }
    __syncthreads();
}

// the LDS image of an upper-round launch: rows (the 1.0 slot's index) and entries it holds
struct Img {
    int R, CAP;
};
// leading outside-term counts of the upper rounds' rows (DFactor::ufold): [2 (row - row0) + bwd]
struct UFold {
    const int16_t *p = nullptr;
    const int16_t *s = nullptr;  // DFactor::ustep, same layout
    int32_t row0 = 0;
    const int16_t *cf = nullptr, *cb = nullptr;  // DFactor::ucode, forward / backward
    uint32_t cf0 = 0, cb0 = 0;
};
// the image of a launch over blocks [b0, b1): their largest row count and entry count (either
// direction), capped by the kernel's R / CAP.  A smaller image than the kernel's maximum lets
// more workgroups share a CU's LDS (the +-64 window's first upper round: 5 per CU instead of 4)
static Img launch_img(const DFactor &F, int64_t b0, int64_t b1, int rmax, int capmax) {
    auto it = F.img_cache.find({b0, b1});
    if (it == F.img_cache.end()) {
        int R = 1, CAP = 1;
        for (int64_t b = b0; b < b1; b++) {
            const int32_t *m = &F.hmeta[(size_t)b * 8];
            R = std::max(R, m[1] - m[0]), CAP = std::max({CAP, m[5] - m[4], m[7] - m[6]});
        }
        it = F.img_cache.emplace(std::make_pair(b0, b1), std::make_pair(R, CAP)).first;
    }
    return Img{std::min(it->second.first, rmax), std::min(it->second.second, capmax)};
}
static size_t img_bytes(const Img &g) { return sweep_lds_bytes(g.R, g.CAP); }
static inline UFold ufold_of(const DFactor &F) {
    const bool cs = F.ustep.n && F.ucode[0].n && F.ucode[1].n;
    return UFold{F.ufold.n ? F.ufold.p : nullptr, cs ? F.ustep.p : nullptr, F.urow0, cs ? F.ucode[0].p : nullptr,
                 cs ? F.ucode[1].p : nullptr, F.ucode0[0], F.ucode0[1]};
}

// The column sweep (one wave; forward and backward alike): the block's rows in the order of
// their keys -- step t solves the row of step t, and since every row's entries are stored in key
// order (forward ascending, backward descending), each row meets its in-block terms at
// increasing steps, all before its own.  Lane L holds the rows of steps L, L + 64, ... (RPL per
// lane) with their accumulators in registers.  Step t broadcasts the finished value of its row
// from the owning lane (v_readlane, no LDS), and every row takes at most ONE term per step: its
// next term if that is column t, or if it is an outside term (a staged product against the 1.0
// slot: column R), which any step may take.  So a step has no branches and no data-dependent
// register shifts: per row a compare, a select, a multiply-subtract and the load of the row's next
// entry, whose LDS latency the next step's broadcast and the other rows cover.  mark_dataflow
// checks per block that this schedule is complete -- every in-block term found at its own step,
// every outside term behind it taken before the row's next in-block term and before the row's own
// step -- and keeps the other loops for a block that fails.  A dense chain (a separator clique: a
// level per row) costs a step per row instead of a level-loop or dataflow trip per row.  Staged
// for it: lv[t] = the local row of step t, c[e] = the step of an in-block column (R: outside).
// DRAIN (blocks whose rows hold outside terms between in-block ones that the steps cannot absorb
// one at a time -- the +-64 window's forward separator rows): a row takes only in-block terms at
// the steps, and right after one it takes the run of outside terms behind it.  The run's length
// is in the in-block entry's staged column (DFactor::ucode, counted at layout), so a drain issues
// its values' loads four at a time, with no LDS round trip per term.
// Same terms, same order; an outside term subtracts v * 1.0 = v: bit-identical.
__device__ __forceinline__ double lane_bcast(double v, int lane) {  // lane: wave-uniform
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
// the sweep's per-row state (registers): accumulator, next entry (staged column c, value v), its
// index e and the row's end e1
template <int RPL>
struct ColState {
    double acc[RPL], v[RPL];
    int e[RPL], e1[RPL], c[RPL], k[RPL];
};
// the outside runs behind this step's in-block terms (k[q] terms of row q >= Q0), four loads per
// row in flight per trip, subtracted in the row's order
template <int Q, int RPL>
__device__ __forceinline__ void colsweep_run_load(const ColState<RPL> &st, const SweepLds &S, int j0, double (&u)[4][4]) {
    if constexpr (Q < RPL) {
        // one base per row and trip, clamped to the run's end (e + k <= e1 <= ne: the four reads
        // stay inside the padded image), the four loads at immediate offsets (two ds_read2_b64)
        const double *b = S.v + st.e[Q] + min(j0, st.k[Q]);
#pragma unroll
        for (int i = 0; i < 4; i++) u[Q][i] = b[i];
    }
}
template <int Q, int RPL>
__device__ __forceinline__ void colsweep_run_sub(ColState<RPL> &st, int j0, const double (&u)[4][4]) {
    if constexpr (Q < RPL) {
        // a term past the run subtracts +0.0: acc - 0.0 == acc, the sign of a zero acc included
        const int kk = st.k[Q] - j0;
#pragma unroll
        for (int i = 0; i < 4; i++) st.acc[Q] = st.acc[Q] - (i < kk ? u[Q][i] : 0.0);
    }
}
template <int Q, int RPL>
__device__ __forceinline__ void colsweep_next_load(const ColState<RPL> &st, const SweepLds &S, int (&cn)[4], double (&vn)[4]) {
    if constexpr (Q < RPL) {
        const int e = st.e[Q] + st.k[Q];
        cn[Q] = (uint16_t)S.c[e], vn[Q] = S.v[e];
    }
}
// a trip issues every row's four loads before its subtractions; the rows' next entries (behind
// their runs) are loaded first, in flight across the trips
template <int Q0, int RPL>
__device__ __forceinline__ void colsweep_drain(ColState<RPL> &st, const SweepLds &S) {
    static_assert(RPL <= 4, "four rows per lane at most");
    int cn[4];
    double vn[4];
    colsweep_next_load<Q0, RPL>(st, S, cn, vn);
    colsweep_next_load<Q0 + 1, RPL>(st, S, cn, vn);
    colsweep_next_load<Q0 + 2, RPL>(st, S, cn, vn);
    colsweep_next_load<Q0 + 3, RPL>(st, S, cn, vn);
    int km = 0;
#pragma unroll
    for (int q = Q0; q < RPL; q++) km = max(km, st.k[q]);
    // (a #pragma unroll loop over the rows inside the trip loop is not unrolled by this compiler)
    for (int j0 = 0; __any(j0 < km); j0 += 4) {
        double u[4][4];
        colsweep_run_load<Q0, RPL>(st, S, j0, u);
        colsweep_run_load<Q0 + 1, RPL>(st, S, j0, u);
        colsweep_run_load<Q0 + 2, RPL>(st, S, j0, u);
        colsweep_run_load<Q0 + 3, RPL>(st, S, j0, u);
        colsweep_run_sub<Q0, RPL>(st, j0, u);
        colsweep_run_sub<Q0 + 1, RPL>(st, j0, u);
        colsweep_run_sub<Q0 + 2, RPL>(st, j0, u);
        colsweep_run_sub<Q0 + 3, RPL>(st, j0, u);
    }
#pragma unroll
    for (int q = Q0; q < RPL; q++) {
        st.e[q] += st.k[q];
        st.c[q] = cn[q], st.v[q] = vn[q];
    }
}
// steps Q * 64 .. (the rows lane + Q * 64 broadcast), rows q >= Q taking terms
template <int Q, int RPL, bool DRAIN>
__device__ __forceinline__ void colsweep_steps(ColState<RPL> &st, const SweepLds &S, int nr) {
    if constexpr (Q < RPL) {
        const int jn = min(kWave, nr - Q * kWave);
        for (int jj = 0; jj < jn; jj++) {
            const int t = Q * kWave + jj;
            const double x = lane_bcast(st.acc[Q], jj);  // the row of step t: every term taken
#pragma unroll
            for (int q = Q; q < RPL; q++) {
                const bool in = (st.c[q] & kCsStep) == t;
                if (DRAIN) {
                    const bool tk = in && st.e[q] < st.e1[q];
                    st.acc[q] = tk ? st.acc[q] - st.v[q] * x : st.acc[q];
                    st.e[q] += tk ? 1 : 0;
                    st.k[q] = tk ? min((st.c[q] >> 8) & kCsRunMax, st.e1[q] - st.e[q]) : 0;
                } else {  // an outside term at the head: taken by any step
                    const bool tk = (in || (st.c[q] & kCsOut)) && st.e[q] < st.e1[q];
                    const double xs = in ? x : 1.0;
                    st.acc[q] = tk ? st.acc[q] - st.v[q] * xs : st.acc[q];
                    st.e[q] += tk ? 1 : 0;
                    st.c[q] = (uint16_t)S.c[st.e[q]], st.v[q] = S.v[st.e[q]];
                }
            }
            if (DRAIN) colsweep_drain<Q, RPL>(st, S);
        }
        colsweep_steps<Q + 1, RPL, DRAIN>(st, S, nr);
    }
}
template <int RPL, bool DRAIN>
__device__ __forceinline__ void levels_colsweep(SweepLds &S, int nr, int lane) {
    ColState<RPL> st;
#pragma unroll
    for (int q = 0; q < RPL; q++) {
        const int t = lane + q * kWave;
        const int k = t < nr ? S.lv[t] : 0;
        st.e[q] = t < nr ? S.ps[k] : 0, st.e1[q] = t < nr ? S.p[k + 1] : 0, st.k[q] = 0;
        st.acc[q] = S.w[k];
        st.c[q] = (uint16_t)S.c[st.e[q]], st.v[q] = S.v[st.e[q]];  // e <= e1 <= ne: inside the padded image
    }
    colsweep_steps<0, RPL, DRAIN>(st, S, nr);
#pragma unroll
    for (int q = 0; q < RPL; q++) {
        const int t = lane + q * kWave;
        if (t < nr) S.w[S.lv[t]] = st.acc[q];
    }
}
__device__ __forceinline__ void colsweep_dispatch(SweepLds &S, int nr, int lane, bool drain) {
    if (drain) {
        if (nr <= kWave) levels_colsweep<1, true>(S, nr, lane);
        else if (nr <= 2 * kWave) levels_colsweep<2, true>(S, nr, lane);
        else levels_colsweep<4, true>(S, nr, lane);
    } else {
        if (nr <= kWave) levels_colsweep<1, false>(S, nr, lane);
        else if (nr <= 2 * kWave) levels_colsweep<2, false>(S, nr, lane);
        else levels_colsweep<4, false>(S, nr, lane);
    }
}

// The level phase, out of LDS.  Per level every thread takes whole rows and consumes a row's
// entries four at a time without branches: the (col, val) arrays are padded by four entries,
// absent terms subtract +0.0 (which leaves every bit of the accumulator unchanged) and the
// selects replace predicated loads, so a row costs a handful of instructions.  The terms are
// still subtracted one at a time in the reference's order.  skip_first: the first level holds
// only rows without entries (their values are already in place), as in round 0 forward.
// PS: rows start at ps[k] (after fold_prefix) instead of p[k].
// ONE: outside-block terms are staged against the 1.0 slot w[R] (column R, value pre-multiplied:
// an exact product) and the padding after the block's entries holds column R, so every column
// read is a valid LDS index and the loop needs no select on the column.
template <int TPB, bool BWD, bool PS = false, int CH = 4, bool WAVE = false, bool ONE = false>
__device__ __forceinline__ void sweep_levels(SweepLds &S, int nl, bool skip_first = false, int tid = -1) {
    if (tid < 0) tid = threadIdx.x;
    static_assert(CH <= kSweepPad, "chunk wider than the padding");
    int l = BWD ? nl - 1 : 0;
    int li0 = 0;
    if (skip_first && !BWD) l = 1, li0 = 1;
    if (li0 >= nl) return;
    int a = S.lv[l], z = S.lv[l + 1];
    for (int li = li0; li < nl; li++) {
        const int ln = BWD ? l - 1 : l + 1;
        int an = 0, zn = 0;
        if (li + 1 < nl) an = S.lv[ln], zn = S.lv[ln + 1];
        for (int k = a + tid; k < z; k += TPB) {
            const int e1 = S.p[k + 1];
            double acc = S.w[k];
            for (int e = PS ? S.ps[k] : S.p[k]; e < e1; e += CH) {
                int c[CH];
                double v[CH], x[CH];
#pragma unroll
                for (int j = 0; j < CH; j++) c[j] = S.c[e + j], v[j] = S.v[e + j];
                if (ONE) {
#pragma unroll
                    for (int j = 0; j < CH; j++) x[j] = S.w[c[j]];
#pragma unroll
                    for (int j = 0; j < CH; j++) acc -= (e + j < e1) ? v[j] * x[j] : 0.0;
                } else {
#pragma unroll
                    for (int j = 0; j < CH; j++) x[j] = S.w[(c[j] >= 0 && e + j < e1) ? c[j] : 0];
#pragma unroll
                    for (int j = 0; j < CH; j++) {
                        const double t = (c[j] >= 0) ? v[j] * x[j] : v[j];
                        acc -= (e + j < e1) ? t : 0.0;
                    }
                }
            }
            S.w[k] = acc;
        }
        if (WAVE) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: LDS in program order
        else __syncthreads();
        l = ln, a = an, z = zn;
    }
}

// The level phase of the persistent round-0 kernel with rows OWNED by lanes: lane tid owns the
// block rows tid + j * TPB (j < RPT) and holds their entry ranges and accumulators in registers
// from the start of the phase, so a level costs the gathers of its rows' terms and one store,
// without first reading each row's bounds and value from LDS (sweep_levels walks row a + tid of
// each level and reads them per level).  Rows are contiguous by level, so a level's rows are the
// owned rows inside [lv[l], lv[l + 1]).  Same terms, same order, same chunking against the 1.0
// slot as sweep_levels<..., ONE>: bit-identical.
// A one-wave workgroup (TPB = 64) needs no barrier between levels: a wave's LDS operations are
// processed in issue order, so the next level's gathers read this level's stores; only the
// compiler must keep the order (a memory clobber), and no s_waitcnt drains the stores first.
// CPK_LEVEL_OWN (A/B builds): 0 sweep_levels, 1 owned rows with a barrier per level, 2 owned
// rows, one-wave levels without it.
#ifndef CPK_LEVEL_OWN
#define CPK_LEVEL_OWN 2
#endif

template <int TPB, int RPT, bool BWD, int CH>
__device__ __forceinline__ void levels_owned(SweepLds &S, int nl, int nr, bool skip_first, int tid) {
    static_assert(CH <= kSweepPad, "chunk wider than the padding");
    uint32_t pe[RPT];  // e0 | e1 << 16 of each owned row
    double acc[RPT];
#pragma unroll
    for (int j = 0; j < RPT; j++) {
        const int k = tid + j * TPB;
        pe[j] = 0u, acc[j] = 0.0;
        if (k < nr) pe[j] = (uint32_t)(uint16_t)S.p[k] | ((uint32_t)(uint16_t)S.p[k + 1] << 16), acc[j] = S.w[k];
    }
    int li0 = 0;
    if (skip_first && !BWD) li0 = 1;
    for (int li = li0; li < nl; li++) {
        const int l = BWD ? nl - 1 - li : li;
        const int a = S.lv[l], z = S.lv[l + 1];
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const int k = tid + j * TPB;
            if (k >= a && k < z) {
                double ac = acc[j];
                const int e1 = (int)(pe[j] >> 16);
                for (int e = (int)(pe[j] & 0xffffu); e < e1; e += CH) {
                    int c[CH];
                    double v[CH], x[CH];
#pragma unroll
                    for (int i = 0; i < CH; i++) c[i] = S.c[e + i], v[i] = S.v[e + i];
#pragma unroll
                    for (int i = 0; i < CH; i++) x[i] = S.w[c[i]];
#pragma unroll
                    for (int i = 0; i < CH; i++) ac -= (e + i < e1) ? v[i] * x[i] : 0.0;
                }
                S.w[k] = ac;
            }
        }
        if (CPK_LEVEL_OWN >= 2 && TPB == kWave) asm volatile("" ::: "memory");
        else __syncthreads();
    }
}

// Forward levels of the persistent round-0 kernel (one 64-lane wave) with lane GROUPS per row.
// Round 0's deep forward levels hold 1-4 rows of ~9-13 terms each (the S fill of a subtree's
// top), which one lane per row walks two terms per pair of dependent LDS trips, while the other
// lanes idle.  A level of nr <= 16 rows instead gives each row a group of G = 16, 8 or 4 lanes
// (within one 16-lane DPP row): lane j of the group forms the product of the row's term c0 + j,
// all at once, and the group's first lane subtracts them in the row's order, shifted to it one
// lane at a time by DPP row_shl:1 (lanes past the row's end contribute 0.0 -- an exact no-op,
// as the padded chunks of sweep_levels).  Wider levels keep one lane per row.  Same products,
// same subtraction order: bit-identical.
#ifndef CPK_LEVEL_GROUP
#define CPK_LEVEL_GROUP 1
#endif
// The same grouping in the upper-round and last-round kernels' one-wave levels, per direction:
// bit-identical either way.  Both on measured slower (S10 backward 0.1835 vs 0.1778 ms,
// profiles/r03_upper_group_ab_v9.txt); CPK_UPPER_GROUP_FWD / _BWD select each (A/B builds).
#ifndef CPK_UPPER_GROUP_FWD
#define CPK_UPPER_GROUP_FWD 0
#endif
#ifndef CPK_UPPER_GROUP_BWD
#define CPK_UPPER_GROUP_BWD 0
#endif
#define CPK_UPPER_GROUP(bwd) ((bwd) ? CPK_UPPER_GROUP_BWD : CPK_UPPER_GROUP_FWD)
__device__ __forceinline__ double row_next_lane(double x) {  // lane i + 1 of its 16-lane row (15: 0)
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x101, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x101, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

// BWD: levels in reverse; PS: rows start at ps[k] (after fold_prefix) instead of p[k]
template <int CH, bool BWD = false, bool PS = false>
__device__ __forceinline__ void levels_grouped(SweepLds &S, int nl, bool skip_first, int lane) {
    for (int li = (skip_first && !BWD) ? 1 : 0; li < nl; li++) {
        const int l = BWD ? nl - 1 - li : li;
        const int a = S.lv[l], z = S.lv[l + 1], nr = z - a;
        if (nr > 16) {  // one lane per row, two terms per LDS round trip (sweep_levels)
            for (int k = a + lane; k < z; k += kWave) {
                const int e1 = S.p[k + 1];
                double acc = S.w[k];
                for (int e = PS ? S.ps[k] : S.p[k]; e < e1; e += CH) {
                    int c[CH];
                    double v[CH], x[CH];
#pragma unroll
                    for (int j = 0; j < CH; j++) c[j] = S.c[e + j], v[j] = S.v[e + j];
#pragma unroll
                    for (int j = 0; j < CH; j++) x[j] = S.w[c[j]];
#pragma unroll
                    for (int j = 0; j < CH; j++) acc -= (e + j < e1) ? v[j] * x[j] : 0.0;
                }
                S.w[k] = acc;
            }
        } else {
            const int lg = nr <= 4 ? 4 : (nr <= 8 ? 3 : 2);  // log2 G
            const int G = 1 << lg, g = lane >> lg, j = lane & (G - 1);
            const bool row = g < nr;
            const int k = a + (row ? g : 0);
            const int e0 = PS ? S.ps[k] : S.p[k], e1 = row ? (int)S.p[k + 1] : e0;
            double acc = S.w[k];
            for (int c0 = 0;; c0 += G) {
                const int e = e0 + c0 + j;
                if (!__any(e0 + c0 < e1)) break;
                const int ec = e < e1 ? e : e0;  // clamped: a valid entry of the block
                const double xv = S.v[ec] * S.w[S.c[ec]];
                double x = e < e1 ? xv : 0.0;
                acc -= x;
                for (int s = 1; s < G; s++) {
                    x = row_next_lane(x);
                    acc -= x;
                }
            }
            if (row && j == 0) S.w[k] = acc;
        }
        asm volatile("" ::: "memory");  // one wave: LDS in issue order (levels_owned)
    }
}
template <int CH>
__device__ __forceinline__ void levels_grouped_fwd(SweepLds &S, int nl, bool skip_first, int lane) {
    levels_grouped<CH, false, false>(S, nl, skip_first, lane);
}

// Dataflow level phase of the upper rounds (one wave, after fold_prefix; terms against the 1.0
// slot R as in sweep_levels<..., ONE>).  The level loop waits, per level, for the slowest row of
// the level, and a row of many in-block terms costs a chunk round trip pair per CH terms in
// every level it sits on.  Here lane L owns the block's rows L, L + 64, ... (forward; backward
// from the last row down), in the order the rows depend on each other, and each iteration it
// takes the next CH terms of its current row, reads their columns' ready flags and values, and
// subtracts the longest READY prefix of them in the row's order; a finished row publishes its
// value and flag and the lane moves on.  No level structure is needed: a row starts on its
// early terms while later ones are still being solved, so a chain of dense rows (a separator
// clique) advances about one row per iteration instead of one level per row-length of chunks.
// Same terms in the same order, not-taken ones subtract +0.0 (an exact no-op): bit-identical.
// The flags live in the level-bound array (lv, R + 1 entries: rows < nr, and R ready), unused
// here.  One wave, so LDS operations complete in issue order: a flag read after a store sees
// it, and a flag is stored after its value.  Progress: the lowest unfinished row (highest,
// backward) has every source done and is its lane's current row, so every iteration takes at
// least one term or finishes a row; `ne + 2` iterations bound the loop (a hang is impossible
// even on malformed input).
// Rows with no terms left are ready from the start; a lane walks only its rows with terms, a
// bit mask of them in a register (next row: lowest set bit), so a finished row hands over to the
// next one without a loop.
template <bool BWD, int CH, bool PS, int RPL>  // PS: rows start at ps[k] (after fold_prefix), else p[k];
                                               // RPL: rows per lane (R / 64)
__device__ __forceinline__ void levels_dataflow(SweepLds &S, int nr, int R, int ne, int lane) {
    static_assert(CH <= kSweepPad, "chunk wider than the padding");
    static_assert(RPL <= 32, "row mask of 32 bits");
    int16_t *rdy = S.lv;
    uint32_t mask = 0;  // bit j: row lane + 64 j has terms to take
#pragma unroll
    for (int j = 0; j < RPL; j++) {
        const int i = lane + j * kWave;
        if (i < nr) {
            const int k = BWD ? nr - 1 - i : i;
            const bool has = (PS ? S.ps[k] : S.p[k]) < S.p[k + 1];
            rdy[k] = has ? 0 : 1;
            mask |= (uint32_t)has << j;
        }
    }
    if (lane == 0) rdy[R] = 1;
    asm volatile("" ::: "memory");
    int k = 0, e = 0, e1 = 0;
    double acc = 0.0;
    auto next_row = [&]() {
        const int i = lane + (int)__builtin_ctz(mask) * kWave;
        k = BWD ? nr - 1 - i : i, e = PS ? S.ps[k] : S.p[k], e1 = S.p[k + 1], acc = S.w[k];
    };
    if (mask) next_row();
    for (int it = 0; it < ne + 2 && __any(mask != 0); it++) {
        if (mask) {
            int c[CH];
            double v[CH], x[CH];
            int16_t f[CH];
#pragma unroll
            for (int j = 0; j < CH; j++) c[j] = S.c[e + j], v[j] = S.v[e + j];
#pragma unroll
            for (int j = 0; j < CH; j++) f[j] = rdy[c[j]], x[j] = S.w[c[j]];
            // ready bits of the chunk's terms, every flag used: no load is sunk into a branch, so
            // all flag and value reads of an iteration are in flight together
            uint32_t rb = 0;
#pragma unroll
            for (int j = 0; j < CH; j++) rb |= (uint32_t)((f[j] != 0) & (e + j < e1)) << j;
            const int t = __builtin_ctz(~rb);  // the leading ready terms
#pragma unroll
            for (int j = 0; j < CH; j++) acc -= j < t ? v[j] * x[j] : 0.0;
            e += t;
            if (e >= e1) {  // row done: publish it, take the next row with terms
                S.w[k] = acc;
                rdy[k] = 1;
                mask &= mask - 1;
                if (mask) next_row();
            }
        }
        asm volatile("" ::: "memory");
    }
}

// Backward write-back of row k (schedule order) with value z:
//   out != null: out[perm[k]] = z, or (ADD) base + z with base = ys[k] when ys is given (the
//                previous solution kept in schedule order), else out[perm[k]];
//   out == null: the solution stays in schedule order (w), and (ADD) ys[k] += z in place.
template <bool ADD>
__device__ __forceinline__ void bwd_store(double *out, double *ys, const int32_t *perm, int64_t k, double z) {
    if (out) {
        const int32_t dst = perm[k];
        out[dst] = ADD ? (ys ? ys[k] : out[dst]) + z : z;
    } else if (ADD) {
        ys[k] = ys[k] + z;
    }
}

template <int TPB>
__global__ __launch_bounds__(TPB) void sptrsv_fwd_kernel(
    int64_t blk0, int R, int CAP, int skip_first, const int32_t *__restrict__ blk_lvl, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    const int32_t *__restrict__ perm, const double *__restrict__ xin, int64_t neg_from, double *w,
    const int *run, const int *active, int sched_in, double *xs) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (skip(run, active)) return;
    const int64_t b = blk0 + blockIdx.x;
    const int l0 = blk_lvl[b], l1 = blk_lvl[b + 1];
    const int r0 = lvl_row[l0], r1 = lvl_row[l1];
    const uint32_t e0 = ptr[r0], e1 = ptr[r1];
    const int nr = r1 - r0, ne = (int)(e1 - e0);
    const int tid = threadIdx.x;
    if (nr <= R && ne <= CAP) {
        SweepLds S(smem, R, CAP);
#pragma unroll 4
        for (int i = tid; i < nr; i += TPB) {
            S.p[i] = (int16_t)(ptr[r0 + i] - e0);
            const int32_t src = sched_in ? r0 + i : perm[r0 + i];
            const double x = xin[src];
            S.w[i] = (src >= neg_from) ? -x : x;
            if (xs) xs[r0 + i] = S.w[i];
        }
        if (tid == 0) S.p[nr] = (int16_t)ne;
        for (int l = tid; l <= l1 - l0; l += TPB) S.lv[l] = (int16_t)(lvl_row[l0 + l] - r0);
#pragma unroll 4
        for (int e = tid; e < ne; e += TPB) {
            const int32_t c = __builtin_nontemporal_load(col + e0 + e);  // streamed once per sweep
            const double v = __builtin_nontemporal_load(val + e0 + e);
            const bool local = c >= r0 && c < r1;
            S.c[e] = local ? (int16_t)(c - r0) : (int16_t)-1;
            S.v[e] = local ? v : v * w[c];
        }
        __syncthreads();
        if (skip_first) {
            sweep_levels<TPB, false>(S, l1 - l0, true);  // round 0: no outside references
        } else {
            fold_prefix<TPB>(S, nr);
            sweep_levels<TPB, false, true, 8>(S, l1 - l0);
        }
        for (int i = tid; i < nr; i += TPB) w[r0 + i] = S.w[i];
        return;
    }
    for (int l = l0; l < l1; l++) {  // direct path: oversized block
        const int a = lvl_row[l], z = lvl_row[l + 1];
        for (int k = a + tid; k < z; k += TPB) {
            const int32_t src = sched_in ? k : perm[k];
            double acc = xin[src];
            if (src >= neg_from) acc = -acc;
            if (xs) xs[k] = acc;
            const uint32_t q1 = ptr[k + 1];
            for (uint32_t e = ptr[k]; e < q1; e++) acc -= val[e] * w[col[e]];
            w[k] = acc;
        }
        __syncthreads();
    }
}

template <int TPB, bool ADD>
__global__ __launch_bounds__(TPB) void sptrsv_bwd_kernel(
    int64_t blk0, int R, int CAP, const int32_t *__restrict__ blk_lvl, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ D, const int32_t *__restrict__ perm, double *w, double *out, const int *run,
    const int *active, double *ys) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (skip(run, active)) return;
    const int64_t b = blk0 + blockIdx.x;
    const int l0 = blk_lvl[b], l1 = blk_lvl[b + 1];
    const int r0 = lvl_row[l0], r1 = lvl_row[l1];
    const uint32_t e0 = ptr[r0], e1 = ptr[r1];
    const int nr = r1 - r0, ne = (int)(e1 - e0);
    const int tid = threadIdx.x;
    if (nr <= R && ne <= CAP) {
        SweepLds S(smem, R, CAP);
#pragma unroll 4
        for (int i = tid; i < nr; i += TPB) {
            S.p[i] = (int16_t)(ptr[r0 + i] - e0);
            S.w[i] = w[r0 + i] / D[r0 + i];
        }
        if (tid == 0) S.p[nr] = (int16_t)ne;
        for (int l = tid; l <= l1 - l0; l += TPB) S.lv[l] = (int16_t)(lvl_row[l0 + l] - r0);
#pragma unroll 4
        for (int e = tid; e < ne; e += TPB) {
            const int32_t c = __builtin_nontemporal_load(col + e0 + e);  // streamed once per sweep
            const double v = __builtin_nontemporal_load(val + e0 + e);
            const bool local = c >= r0 && c < r1;
            S.c[e] = local ? (int16_t)(c - r0) : (int16_t)-1;
            S.v[e] = local ? v : v * w[c];
        }
        __syncthreads();
        fold_prefix<TPB>(S, nr);
        sweep_levels<TPB, true, true, 8>(S, l1 - l0);
        for (int i = tid; i < nr; i += TPB) {
            const double z = S.w[i];
            w[r0 + i] = z;
            bwd_store<ADD>(out, ys, perm, r0 + i, z);
        }
        return;
    }
    for (int l = l1 - 1; l >= l0; l--) {  // direct path: oversized block
        const int a = lvl_row[l], z = lvl_row[l + 1];
        for (int k = a + tid; k < z; k += TPB) {
            double acc = w[k] / D[k];
            const uint32_t q1 = ptr[k + 1];
            for (uint32_t e = ptr[k]; e < q1; e++) acc -= val[e] * w[col[e]];
            w[k] = acc;
            bwd_store<ADD>(out, ys, perm, k, acc);
        }
        __syncthreads();
    }
}

// ---- persistent, software-pipelined sweep for the wide round 0 -------------------------------
// Round 0 holds ~all rows in tens of thousands of small blocks.  A block's life is HBM latency
// (staging) followed by LDS latency (levels), and LDS caps residency, so each workgroup here
// walks a strided list of blocks and overlaps them: while block b runs its levels out of LDS,
// the independent loads of block b + G (row pointers, perm, level bounds, entries) are already
// in flight into registers.  Only the dependent gathers (x[perm] forward, w[col] of rows in
// later rounds backward) stay exposed.  Per-block metadata is one 32-byte record (scalar load).
// Arithmetic and order are those of the one-block-per-workgroup kernels: bit-identical.
struct BlkMeta {
    int32_t r0, r1, l0, l1, fe0, fe1, be0, be1;
};

// Fused refinement residual (RES): the forward sweep's input r = xs - Kps*y for the block's rows,
// formed inside the sweep instead of by a residual SpMV launch (opLDL2.m:175-182, one refinement
// step).  Kps, y and xs are in schedule order, so a block's Kps rows are one contiguous entry
// range: the entries are streamed coalesced (prefetched with the block), the products staged in
// the block's entry region of LDS, and each row summed in Kps's column order from 0.0, then
// subtracted from xs: the operations of spmv_stream<EpiResidSched>, bit for bit.
struct ResArgs {
    const uint32_t *ptr = nullptr;  // Kps rows
    const int32_t *col = nullptr;
    const double *val = nullptr;
    const double *y = nullptr;   // the current solution in schedule order
    const double *xs = nullptr;  // the signed input in schedule order
    // rows [tail0, tail1) above round 0: r (into w) by the workgroups once their blocks are done,
    // one row per lane, entries summed in order from 0.0 (the residual SpMV's row, without a launch)
    int64_t tail0 = 0, tail1 = 0;
};

// Distributed payloads packed by the sweeps' write-back instead of a gather launch:
//   forward: the separator exchange's payload -- slot[schedule row] (-1: not sent) -> buf, and
//            (workgroup 0 of the round-0 launch) rank 0's T inputs +-x[tdof] and the piggyback
//            values: what tpack_kernel writes;
//   backward: the residual SpMV's Kp halo -- slot[output index] -> buf, the value written to
//            the output: what launch_halo's gather writes.
__device__ __forceinline__ void pack_put(const PackArgs &pk, int64_t key, double z) {
    if (pk.slot) {
        const int32_t s = pk.slot[key];
        if (s >= 0) pk.buf[s] = z;
    }
}
// one T input per thread of the launch (thread e of the grid), so no workgroup is delayed by
// more than one dependent load pair; the piggyback values by the first threads of workgroup 0
__device__ __forceinline__ void pack_inputs(const PackArgs &pk, int64_t e) {
    if (!pk.buf) return;
    if (e < pk.ntdof) {
        const int32_t d = pk.tdof[e];
        const double v = pk.x[d];
        pk.buf[pk.nsend + e] = d >= pk.neg_from ? -v : v;
    }
    if (pk.piggy && e < (int64_t)kSepPiggy) pk.buf[pk.kt_data + e] = pk.piggy[e];
}

// ---- upper rounds ------------------------------------------------------------------------------
// One workgroup per block, as sptrsv_fwd_kernel / sptrsv_bwd_kernel, with the staging laid out
// for memory-level parallelism: the block's 32-byte record is one scalar load, every thread
// issues all of its row and entry loads at once, then all of its gathers (input through perm,
// w of outside-block columns) with clamped, unconditional addresses, so staging costs about two
// dependent round trips instead of one per predicated slot.  Fold and levels as before.
#ifdef CPK_PIPE_STAMPS
// per-block cycles (s_memtime) of the last launch of each unsplit round-0 variant: [fwd, fwd +
// fused residual, bwd, bwd accumulating][block] (tools/blk_cycles.py: the round-0 cost model),
// then the upper rounds' phases [fwd, bwd][staging, fold, levels, write-back][block]
// (tools/upper_cycles.py)
constexpr int kBlkCycMax = 1 << 20;  // round 0: keyed by the block's first level (BlkMeta::l0)
__device__ uint64_t g_blk_cyc[12 * kBlkCycMax];
#define CPK_UP_STAMP(k)                                                                          \
    do {                                                                                       \
        const uint64_t t_ = (uint64_t)clock64();                                               \
        if (threadIdx.x == 0 && b < kBlkCycMax) g_blk_cyc[(4 + (BWD ? 4 : 0) + (k)) * kBlkCycMax + b] = t_ - tp; \
        tp = t_;                                                                               \
    } while (0)
#else
#define CPK_UP_STAMP(k) (void)0
#endif
// one block of an upper round (the body of sptrsv_upper_kernel); ends with the block's write-back
// SC (the chain kernel): w is handed between blocks of one launch, so every w value a block may
// read from another block, and every w value it writes, goes through agent-scope (sc1) loads and
// stores (MI355X_MICROARCH.md "Valid forms", row 1), never through this CU's L1
template <bool SC>
__device__ __forceinline__ double wld(const double *p) {
    if constexpr (SC) return ld_agent(p);
    return *p;
}
template <bool SC>
__device__ __forceinline__ void wst(double *p, double v) {
    if constexpr (SC) st_agent(p, v);
    else *p = v;
}
// wait (the chain kernel): called by every thread between the block's static loads (row pointers,
// entries, perm, D, level bounds, the forward input) and its loads of w -- a chained task issues
// the former before it polls its producers' flags, so their HBM round trip overlaps the wait
struct NoWait {
    __device__ void operator()() const {}
};
template <int TPB, int RPU, int EPU, bool BWD, bool ADD, bool SC = false, class Wait = NoWait>
__device__ __forceinline__ void upper_block(
    char *smem, const BlkMeta m, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ D, const int32_t *__restrict__ perm, const double *__restrict__ xin, int64_t neg_from,
    double *w, double *out, int sched_in, double *ys, double *xs, const PackArgs &pk, const UFold &uf, int64_t b,
    const Img &img, const Wait &wait = Wait{}) {
    // the LDS image of this launch (Img: its blocks' largest rows / entries, <= the kernel's R / CAP)
    constexpr int RMAX = RPU * TPB;
    const int R = img.R, CAP = img.CAP;
#ifdef CPK_PIPE_STAMPS
    uint64_t tp = (uint64_t)clock64();
#else
    (void)b;
#endif
    const int r0 = m.r0, r1 = m.r1, nr = r1 - r0, nl = (m.l1 & kMetaL1Mask) - m.l0;
    const uint32_t e0 = BWD ? (uint32_t)m.be0 : (uint32_t)m.fe0;
    const int ne = BWD ? m.be1 - m.be0 : m.fe1 - m.fe0;
    const int tid = threadIdx.x;
    // the column sweep for this block and direction (mark_dataflow); it needs the step table
    const bool cs = uf.s != nullptr && (m.l1 & (BWD ? kMetaCsBwd : kMetaCsFwd));
    SweepLds S(smem, R, CAP);
    (void)CAP;
    uint32_t q[RPU];
    int32_t sp[RPU], fo[RPU], st[RPU];
    double a[RPU], d[RPU];
    int32_t c[EPU];
    double v[EPU], g[EPU];
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        const int i = tid + j * TPB, rr = r0 + (i < nr ? i : nr - 1);
        q[j] = ptr[rr], sp[j] = (BWD ? out != nullptr : !sched_in) ? perm[rr] : rr;
        fo[j] = uf.p ? uf.p[2 * (rr - uf.row0) + (BWD ? 1 : 0)] : 0;
        st[j] = cs ? uf.s[2 * (rr - uf.row0) + (BWD ? 1 : 0)] : 0;
        if (BWD) d[j] = D[rr];
    }
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const int e = tid + u * TPB;
        const uint32_t ec = e0 + (uint32_t)(e < ne ? e : 0);
        c[u] = __builtin_nontemporal_load(col + ec), v[u] = __builtin_nontemporal_load(val + ec);
    }
    // staged columns (static: before the wait): local row, or the layout's code (column sweep; lv
    // holds the rows by step); R outside
    int32_t cl[EPU];
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const bool local = c[u] >= r0 && c[u] < r1;
        const uint32_t ec = e0 + (uint32_t)(tid + u * TPB < ne ? tid + u * TPB : 0);
        cl[u] = cs ? (int32_t)(uint16_t)(BWD ? uf.cb[ec - uf.cb0] : uf.cf[ec - uf.cf0]) : (!local ? R : c[u] - r0);
    }
    if (!cs)
        for (int l = tid; l <= nl; l += TPB) S.lv[l] = (int16_t)(lvl_row[m.l0 + l] - r0);
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        if (!BWD) a[j] = xin[sp[j]];
    }
    wait();
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        if (BWD) a[j] = wld<SC>(w + r0 + (tid + j * TPB < nr ? tid + j * TPB : nr - 1));
    }
#pragma unroll
    for (int u = 0; u < EPU; u++) g[u] = wld<SC>(w + ((c[u] >= r0 && c[u] < r1) ? r0 : c[u]));
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        const int i = tid + j * TPB;
        if (i < nr) {
            S.p[i] = (int16_t)(q[j] - e0);
            if (uf.p) S.ps[i] = (int16_t)(q[j] - e0 + fo[j]);
            if (cs) S.lv[st[j]] = (int16_t)i;
            S.w[i] = BWD ? a[j] / d[j] : ((sp[j] >= neg_from) ? -a[j] : a[j]);
            if (!BWD && xs) xs[r0 + i] = S.w[i];
        }
    }
    if (tid == 0) S.p[nr] = (int16_t)ne, S.w[R] = 1.0;
    if (tid < kSweepPad) S.c[ne + tid] = (int16_t)R;
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const int e = tid + u * TPB;
        if (e < ne) {
            const bool local = c[u] >= r0 && c[u] < r1;
            S.c[e] = (int16_t)cl[u];  // outside: R, pre-multiplied against the 1.0 slot
            S.v[e] = local ? v[u] : v[u] * g[u];
        }
    }
    __syncthreads();
    CPK_UP_STAMP(0);
    if (uf.p) fold_known<TPB>(S, nr, tid);
    else fold_prefix<TPB, 1>(S, nr, -1, R);
    CPK_UP_STAMP(1);
    // levels on one wave: a level holds a few rows, and without a workgroup barrier per level
    // (a single wave's LDS accesses complete in program order) the chain is LDS latency only;
    // narrow levels give each row a lane group (levels_grouped)
    if (tid < kWave) {
        if (cs) colsweep_dispatch(S, nr, tid, m.l1 & (BWD ? kMetaCoBwd : kMetaCoFwd));
        else if (CPK_UPPER_DATAFLOW && (m.l1 & (BWD ? kMetaDfBwd : kMetaDfFwd)))
            levels_dataflow<BWD, CPK_DF_CH(BWD), true, RMAX / kWave>(S, nr, R, ne, tid);
        else if (CPK_UPPER_GROUP(BWD)) levels_grouped<CPK_UPPER_CH(BWD), BWD, true>(S, nl, false, tid);
        else sweep_levels<kWave, BWD, true, CPK_UPPER_CH(BWD), true, true>(S, nl, false, tid);
    }
    __syncthreads();
    CPK_UP_STAMP(2);
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        const int i = tid + j * TPB;
        if (i < nr) {
            const double z = S.w[i];
            wst<SC>(w + r0 + i, z);
            if (BWD) {
                if (out) {
                    const double o = ADD ? (ys ? ys[r0 + i] : out[sp[j]]) + z : z;
                    out[sp[j]] = o;
                    pack_put(pk, sp[j], o);
                } else {  // the solution stays in schedule order: packed by schedule row
                    const double o = ADD ? ys[r0 + i] + z : z;
                    if (ADD) ys[r0 + i] = o;
                    pack_put(pk, r0 + i, o);
                }
            } else {
                pack_put(pk, r0 + i, z);
            }
        }
    }
    CPK_UP_STAMP(3);
}

template <int TPB, int RPU, int EPU, bool BWD, bool ADD>
__global__ __launch_bounds__(TPB) void sptrsv_upper_kernel(
    int64_t blk0, const BlkMeta *__restrict__ meta, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ D, const int32_t *__restrict__ perm, const double *__restrict__ xin, int64_t neg_from,
    double *w, double *out, const int *run, const int *active, int sched_in, double *ys, double *xs, PackArgs pk,
    UFold uf, Img img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (skip(run, active)) return;
    upper_block<TPB, RPU, EPU, BWD, ADD>(smem, meta[blk0 + blockIdx.x], lvl_row, ptr, col, val, D, perm, xin, neg_from,
                                         w, out, sched_in, ys, xs, pk, uf, blk0 + blockIdx.x, img);
}

// The last round's forward and backward sweeps in one launch (single GPU).  The sweeps meet at
// the top of the tree: forward rounds 0 .. R-1, then backward R-1 .. 0, so the last round's
// blocks are solved forward and at once backward; a block holds whole subtrees of the last
// remaining tree, so its backward terms stay inside it.  One workgroup per block stages the
// forward and backward entries together (every independent load in flight at once), runs the
// forward fold and levels, divides by D in LDS and runs the backward levels -- the operations of
// sptrsv_upper_kernel forward, its write-back and w / D, and sptrsv_upper_kernel backward, in
// that order: bit-identical, one launch and one staging round trip fewer per solve.
template <int TPB, int RPU, int EPU, bool ADD, bool SC = false, class Wait = NoWait>
__device__ __forceinline__ void last_block(
    char *smem, const BlkMeta m, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ fptr, const int32_t *__restrict__ fcol, const double *__restrict__ fval,
    const uint32_t *__restrict__ bptr, const int32_t *__restrict__ bcol, const double *__restrict__ bval,
    const double *__restrict__ D, const int32_t *__restrict__ perm, const double *__restrict__ xin, int64_t neg_from,
    int sched_in, double *xs, double *w, double *out, double *ys, const UFold &uf, const Img &img,
    const Wait &wait = Wait{}) {
    constexpr int RMAX = RPU * TPB;
    const int R = img.R, CAP = img.CAP;
    const int r0 = m.r0, r1 = m.r1, nr = r1 - r0, nl = (m.l1 & kMetaL1Mask) - m.l0;
    const int nef = m.fe1 - m.fe0, neb = m.be1 - m.be0;
    const int tid = threadIdx.x;
    const bool csf = uf.s != nullptr && (m.l1 & kMetaCsFwd), csb = uf.s != nullptr && (m.l1 & kMetaCsBwd);
    SweepLds S(smem, R, CAP);
    (void)CAP;
    uint32_t qf[RPU], qb[RPU];
    int32_t sp[RPU], dp[RPU], fof[RPU], fob[RPU], stf[RPU], stb[RPU];
    double a[RPU], d[RPU];
    int32_t cf[EPU], cb[EPU];
    double vf[EPU], vb[EPU], g[EPU];
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        const int i = tid + j * TPB, rr = r0 + (i < nr ? i : nr - 1);
        qf[j] = fptr[rr], qb[j] = bptr[rr], d[j] = D[rr];
        fof[j] = uf.p ? uf.p[2 * (rr - uf.row0)] : 0, fob[j] = uf.p ? uf.p[2 * (rr - uf.row0) + 1] : 0;
        stf[j] = csf ? uf.s[2 * (rr - uf.row0)] : 0, stb[j] = csb ? uf.s[2 * (rr - uf.row0) + 1] : 0;
        sp[j] = sched_in ? rr : perm[rr];
        dp[j] = out ? perm[rr] : rr;
    }
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const int e = tid + u * TPB;
        const uint32_t ef = (uint32_t)m.fe0 + (uint32_t)(e < nef ? e : 0);
        cf[u] = __builtin_nontemporal_load(fcol + ef), vf[u] = __builtin_nontemporal_load(fval + ef);
    }
    int32_t cl[EPU];  // staged columns: local row, or the layout's code (column sweep); R outside
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const bool local = cf[u] >= r0 && cf[u] < r1;
        const uint32_t ef = (uint32_t)m.fe0 + (uint32_t)(tid + u * TPB < nef ? tid + u * TPB : 0);
        cl[u] = csf ? (int32_t)(uint16_t)uf.cf[ef - uf.cf0] : (!local ? R : cf[u] - r0);
    }
    if (!csf)
        for (int l = tid; l <= nl; l += TPB) S.lv[l] = (int16_t)(lvl_row[m.l0 + l] - r0);
#pragma unroll
    for (int j = 0; j < RPU; j++) a[j] = xin[sp[j]];
    wait();
    // the backward entries after the wait (held across it, they spilled in the chain kernel);
    // their round trip still overlaps the forward phase
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const int e = tid + u * TPB;
        const uint32_t eb = (uint32_t)m.be0 + (uint32_t)(e < neb ? e : 0);
        cb[u] = __builtin_nontemporal_load(bcol + eb), vb[u] = __builtin_nontemporal_load(bval + eb);
    }
#pragma unroll
    for (int u = 0; u < EPU; u++) g[u] = wld<SC>(w + ((cf[u] >= r0 && cf[u] < r1) ? r0 : cf[u]));
    // ---- forward (sptrsv_upper_kernel<..., false, false>)
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        const int i = tid + j * TPB;
        if (i < nr) {
            S.p[i] = (int16_t)(qf[j] - (uint32_t)m.fe0);
            if (uf.p) S.ps[i] = (int16_t)(qf[j] - (uint32_t)m.fe0 + fof[j]);
            if (csf) S.lv[stf[j]] = (int16_t)i;
            S.w[i] = (sp[j] >= neg_from) ? -a[j] : a[j];
            if (xs) xs[r0 + i] = S.w[i];
        }
    }
    if (tid == 0) S.p[nr] = (int16_t)nef, S.w[R] = 1.0;
    if (tid < kSweepPad) S.c[nef + tid] = (int16_t)R;
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const int e = tid + u * TPB;
        if (e < nef) {
            const bool local = cf[u] >= r0 && cf[u] < r1;
            S.c[e] = (int16_t)cl[u];
            S.v[e] = local ? vf[u] : vf[u] * g[u];
        }
    }
    __syncthreads();
    if (uf.p) fold_known<TPB>(S, nr, tid);
    else fold_prefix<TPB, 1>(S, nr, -1, R);
    if (tid < kWave) {
        if (csf) colsweep_dispatch(S, nr, tid, m.l1 & kMetaCoFwd);
        else if (CPK_UPPER_DATAFLOW && (m.l1 & kMetaDfFwd)) levels_dataflow<false, CPK_DF_CH(false), true, RMAX / kWave>(S, nr, R, nef, tid);
        else if (CPK_UPPER_GROUP(false)) levels_grouped<CPK_UPPER_CH(false), false, true>(S, nl, false, tid);
        else sweep_levels<kWave, false, true, CPK_UPPER_CH(false), true, true>(S, nl, false, tid);
    }
    __syncthreads();
    // ---- backward (sptrsv_upper_kernel<..., true, ADD>): w / D, the entries, fold, levels; the
    // backward terms of a last-round block are its own rows (the 1.0 slot path is kept for any other)
#pragma unroll
    for (int u = 0; u < EPU; u++) g[u] = (tid + u * TPB < neb && (cb[u] < r0 || cb[u] >= r1)) ? wld<SC>(w + cb[u]) : 0.0;
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        const int i = tid + j * TPB;
        if (i < nr) {
            S.w[i] = S.w[i] / d[j];
            S.p[i] = (int16_t)(qb[j] - (uint32_t)m.be0);
            if (uf.p) S.ps[i] = (int16_t)(qb[j] - (uint32_t)m.be0 + fob[j]);
            if (csb) S.lv[stb[j]] = (int16_t)i;
        }
    }
    if (tid == 0) S.p[nr] = (int16_t)neb;
    if (tid < kSweepPad) S.c[neb + tid] = (int16_t)R;
    // the level loop needs the level bounds back if the forward loop took lv (flags or steps)
    if ((csf || (CPK_UPPER_DATAFLOW && (m.l1 & kMetaDfFwd))) && !csb && !(CPK_UPPER_DATAFLOW && (m.l1 & kMetaDfBwd)))
        for (int l = tid; l <= nl; l += TPB) S.lv[l] = (int16_t)(lvl_row[m.l0 + l] - r0);
#pragma unroll
    for (int u = 0; u < EPU; u++) {
        const int e = tid + u * TPB;
        if (e < neb) {
            const bool local = cb[u] >= r0 && cb[u] < r1;
            S.c[e] = csb ? uf.cb[(uint32_t)m.be0 + (uint32_t)e - uf.cb0] : (int16_t)(!local ? R : cb[u] - r0);
            S.v[e] = local ? vb[u] : vb[u] * g[u];
        }
    }
    __syncthreads();
    if (uf.p) fold_known<TPB>(S, nr, tid);
    else fold_prefix<TPB, 1>(S, nr, -1, R);
    if (tid < kWave) {
        if (csb) colsweep_dispatch(S, nr, tid, m.l1 & kMetaCoBwd);
        else if (CPK_UPPER_DATAFLOW && (m.l1 & kMetaDfBwd)) levels_dataflow<true, CPK_DF_CH(true), true, RMAX / kWave>(S, nr, R, neb, tid);
        else if (CPK_UPPER_GROUP(true)) levels_grouped<CPK_UPPER_CH(true), true, true>(S, nl, false, tid);
        else sweep_levels<kWave, true, true, CPK_UPPER_CH(true), true, true>(S, nl, false, tid);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPU; j++) {
        const int i = tid + j * TPB;
        if (i < nr) {
            const double z = S.w[i];
            wst<SC>(w + r0 + i, z);
            if (out) out[dp[j]] = ADD ? (ys ? ys[r0 + i] : out[dp[j]]) + z : z;
            else if (ADD) ys[r0 + i] = ys[r0 + i] + z;
        }
    }
}

template <int TPB, int RPU, int EPU, bool ADD>
__global__ __launch_bounds__(TPB) void sptrsv_last_kernel(
    int64_t blk0, const BlkMeta *__restrict__ meta, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ fptr, const int32_t *__restrict__ fcol, const double *__restrict__ fval,
    const uint32_t *__restrict__ bptr, const int32_t *__restrict__ bcol, const double *__restrict__ bval,
    const double *__restrict__ D, const int32_t *__restrict__ perm, const double *__restrict__ xin, int64_t neg_from,
    int sched_in, double *xs, double *w, double *out, const int *run, const int *active, double *ys, UFold uf,
    Img img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (skip(run, active)) return;
    last_block<TPB, RPU, EPU, ADD>(smem, meta[blk0 + blockIdx.x], lvl_row, fptr, fcol, fval, bptr, bcol, bval, D, perm,
                                   xin, neg_from, sched_in, xs, w, out, ys, uf, img);
}

// the last round fused (fwd + bwd) when it is an upper round whose blocks fit sptrsv_last_kernel
bool fuse_last_ok(const DFactor &F) {
    const int64_t R = (int64_t)F.round_ptr.size() - 1;
    return F.fuse_last && R >= 2 && (F.sweep_threads[1] == 512 || F.sweep_threads[1] == 256) &&
           F.sweep_rows[1] <= 1024 && F.sweep_cap[1] <= 4096 &&
           (int64_t)F.round_fits.size() >= R && F.round_fits[R - 1] && !F.no_upper;
}

static void launch_last(Ctx &c, const DFactor &F, const FwdIn &in, double *w, double *out, bool add,
                        const int *run, const int *active, double *ys) {
    constexpr int TPB = 512, RPU = 2, EPU = 8;
    const int64_t R = (int64_t)F.round_ptr.size() - 1;
    const int64_t b0 = F.round_ptr[R - 1], nb = F.round_ptr[R] - b0;
    if (!nb) return;
    const size_t lds = sweep_lds_bytes(RPU * TPB, EPU * TPB);
    const Img img{RPU * TPB, EPU * TPB};
    static const bool lds_ok = lds <= 64 * 1024 ||
        (hipFuncSetAttribute((const void *)sptrsv_last_kernel<TPB, RPU, EPU, false>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess &&
         hipFuncSetAttribute((const void *)sptrsv_last_kernel<TPB, RPU, EPU, true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess);
    if (!lds_ok) throw Error(CPK_ERR_HIP, "sptrsv_last_kernel: LDS image not admitted");
    const BlkMeta *meta = reinterpret_cast<const BlkMeta *>(F.meta.p);
    if (add)
        hipLaunchKernelGGL((sptrsv_last_kernel<TPB, RPU, EPU, true>), dim3((unsigned)nb), dim3(TPB), img_bytes(img), c.stream, b0,
                           meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p, F.perm.p,
                           in.xin, in.neg_from, in.sched_in, in.xs, w, out, run, active, ys, ufold_of(F), img);
    else
        hipLaunchKernelGGL((sptrsv_last_kernel<TPB, RPU, EPU, false>), dim3((unsigned)nb), dim3(TPB), img_bytes(img), c.stream, b0,
                           meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p, F.perm.p,
                           in.xin, in.neg_from, in.sched_in, in.xs, w, out, run, active, ys, ufold_of(F), img);
    CPK_HIP(hipGetLastError());
}

// ---- the sweep chains ----------------------------------------------------------------------------
// Upper rounds in ONE launch.  kChainFull: forward rounds 1 .. R-2, the last round (forward and
// backward, as sptrsv_last_kernel), backward rounds R-2 .. 1 (single GPU); kChainFwd / kChainBwd:
// forward rounds 1 .. R-1 / backward rounds R-1 .. 1 (distributed: the separator solve sits
// between them).  One workgroup per task, tasks in topological order (blockIdx = task); a task
// waits for its own producers -- the blocks holding the rows its entries read (build_chain) --
// not for the whole previous round, then runs the block exactly as the round kernels do
// (bit-identical) and publishes a done flag.  Deadlock-free without co-residency: workgroups are
// dispatched in blockIdx order (per XCD queue), so every producer of a resident waiter (a smaller
// index) has been dispatched.  Hand-off: MI355X_MICROARCH.md "Valid forms" row 1 -- every w value
// crossing blocks is stored and loaded sc1 (upper_block<SC>), each storing wave drains
// (vmcnt(0)) before the workgroup barrier, one lane stores the flag sc1, and consumers poll it
// sc1.  Flags hold the launch's epoch + 1 (no reset pass); the last workgroup (ticket) advances
// the epoch.  Every spin is bounded: a wait that outlives kChainSpinCap sets the error word, every
// other waiter of that launch then gives up, and the host raises CPK_ERR_HIP (check_chain).
#ifndef CPK_CHAIN_SPIN_CAP
#define CPK_CHAIN_SPIN_CAP (1u << 20)
#endif
constexpr uint32_t kChainSpinCap = CPK_CHAIN_SPIN_CAP;  // polls (2^20: with the back-off below, ~0.5 s)
// The hand-off's envelope (MI355X_MICROARCH.md "Valid forms"): sc1 loads may replace the
// consumer's agent acquire only in a measured table row, and row 1 (one lane per storing
// workgroup signals with an sc1 flag after every storing wave's vmcnt(0) and a barrier; sc1
// 4/8-byte stores and loads; hipMalloc'd memory) holds for ONE workgroup per CU.
// CPK_CHAIN_LDS_MIN (default 83968 bytes, above half of the CU's 160 KB LDS): a floor on the
// chain launch's LDS, so exactly one chain workgroup is resident per CU -- the row's residency.
// CPK_CHAIN_ACQUIRE (default 0): an agent acquire after each task's polls instead (the guide's
// "always" form, needed at several workgroups per CU).  Round 6 A/B (profiles/r06_ab/
// chain_handoff_*_ab.log, three interleaved rounds): +-64 window 469.1 it/s with the acquire at
// four per CU, 470.8 without it at four per CU (outside the envelope: round 5's form), 471.6 at
// one per CU without it; the +-4 window 941-946 for all three.  Both valid forms cost nothing
// measurable; one per CU, no acquire, is the default.
#ifndef CPK_CHAIN_ACQUIRE
#define CPK_CHAIN_ACQUIRE 0
#endif
#ifndef CPK_CHAIN_LDS_MIN
#define CPK_CHAIN_LDS_MIN 83968
#endif
// polling back-off of a waiting task: CPK_CHAIN_FAST_POLLS polls s_sleep CPK_CHAIN_SLEEP0 apart,
// then CPK_CHAIN_SLEEP1 (units of 64 cycles)
#ifndef CPK_CHAIN_FAST_POLLS
#define CPK_CHAIN_FAST_POLLS 16
#endif
#ifndef CPK_CHAIN_SLEEP0
#define CPK_CHAIN_SLEEP0 2
#endif
#ifndef CPK_CHAIN_SLEEP1
#define CPK_CHAIN_SLEEP1 16
#endif
// the rounds a chain covers: the narrow top of the tree (rounds of at most chain_wide blocks,
// and at least two of them).  A wide round's blocks are all ready at once -- a launch of their
// own costs nothing there -- and in a chain hundreds of its blocks would sit polling the few
// flags of the round above: the guide's warning, many pollers cut the chip's bandwidth.
struct ChainArgs {
    const int32_t *task, *dptr, *didx;
    uint32_t *flag, *ctrl;
    int ntask;
};
__device__ __forceinline__ uint32_t ld_agent32(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent32(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int TPB, int RPU, int EPU, bool ADD>
__global__ __launch_bounds__(TPB) void sptrsv_chain_kernel(
    ChainArgs ch, const BlkMeta *__restrict__ meta, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ fptr, const int32_t *__restrict__ fcol, const double *__restrict__ fval,
    const uint32_t *__restrict__ bptr, const int32_t *__restrict__ bcol, const double *__restrict__ bval,
    const double *__restrict__ D, const int32_t *__restrict__ perm, const double *__restrict__ xin, int64_t neg_from,
    int sched_in, double *xs, double *w, double *out, const int *run, const int *active, double *ys, PackArgs pk,
    UFold uf, Img img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ uint32_t s_epoch;
    if (skip(run, active)) return;
    const int t = blockIdx.x;
    if (threadIdx.x == 0) s_epoch = ld_agent32(ch.ctrl);
    __syncthreads();
    const uint32_t want = s_epoch + 1;
    const int32_t task = ch.task[t];
    const int kind = task >> 28, b = task & ((1 << 28) - 1);
    // the producers' flags, polled between the block's static loads and its loads of w
    const int k0 = ch.dptr[t], k1 = ch.dptr[t + 1];
    const int32_t *didx = ch.didx;
    const uint32_t *flag = ch.flag;
    uint32_t *err = ch.ctrl + 2;
    auto wait = [k0, k1, didx, flag, err, want]() {
        for (int k = k0 + (int)threadIdx.x; k < k1; k += TPB) {
            const uint32_t *f = flag + didx[k];
            uint32_t spins = 0;
            while (ld_agent32(f) != want) {
                // a wait of THIS launch timed out somewhere: give up.  The word holds the epoch of
                // the launch that timed out, so a word left set (until the host's next check,
                // check_chain or the distributed solve's status agreement) never disables the
                // waits of a later launch
                if (ld_agent32(err) == want) break;
                if (++spins > kChainSpinCap) {
                    st_agent32(err, want);
                    break;
                }
                // back off: a few quick polls, then ~1000 cycles apart (poll traffic stays low)
                if (spins < CPK_CHAIN_FAST_POLLS) __builtin_amdgcn_s_sleep(CPK_CHAIN_SLEEP0);
                else __builtin_amdgcn_s_sleep(CPK_CHAIN_SLEEP1);
            }
        }
        __syncthreads();
#if CPK_CHAIN_ACQUIRE
        // the consumer's agent acquire after the polls (MI355X_MICROARCH.md "Valid forms":
        // poll -> acquire -> s_waitcnt vmcnt(0) -> barrier -> loads).  The sc1 loads alone replace
        // it only for one workgroup per CU (the table's row 1); this kernel runs up to four
        if (k1 > k0 && threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
#endif
    };
    if (kind == 0)
        upper_block<TPB, RPU, EPU, false, false, true>(smem, meta[b], lvl_row, fptr, fcol, fval, D, perm, xin, neg_from, w,
                                                       nullptr, sched_in, nullptr, xs, pk, uf, b, img, wait);
    else if (kind == 1)
        last_block<TPB, RPU, EPU, ADD, true>(smem, meta[b], lvl_row, fptr, fcol, fval, bptr, bcol, bval, D, perm, xin,
                                             neg_from, sched_in, xs, w, out, ys, uf, img, wait);
    else
        upper_block<TPB, RPU, EPU, true, ADD, true>(smem, meta[b], lvl_row, bptr, bcol, bval, D, perm, nullptr, 0, w, out,
                                                    0, ys, nullptr, pk, uf, b, img, wait);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's w stores done
    __syncthreads();
    if (threadIdx.x == 0) {
        st_agent32(ch.flag + t, want);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__hip_atomic_fetch_add(ch.ctrl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)ch.ntask - 1) {
            st_agent32(ch.ctrl + 1, 0u);
            st_agent32(ch.ctrl, want);  // the next launch's epoch
        }
    }
}

// the distributed solve's status word (solvers.hip, agree_status): a host-side code of this rank
// (0: none) and every sweep chain's device error word of the preconditioner, as one int64 --
// (code << 16) | (0xffff - rank), so the ranks' maximum names the largest code and, among equal
// codes, the lowest failing rank
__global__ void solve_status_kernel(int64_t *out, int64_t host, const uint32_t *e0, const uint32_t *e1,
                                    const uint32_t *e2, const uint32_t *e3, const uint32_t *e4, const uint32_t *e5,
                                    int64_t chain_code) {
    int64_t v = host;
    const uint32_t *e[6] = {e0, e1, e2, e3, e4, e5};
    for (int i = 0; i < 6; i++)
        if (e[i] && ld_agent32(e[i]) != 0) v = max(v, chain_code);
    out[0] = v;
}
void launch_solve_status(Ctx &c, const DFactor *const *F, int nf, int64_t host_code, int64_t chain_code, int64_t *out) {
    const uint32_t *e[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    int k = 0;
    for (int i = 0; i < nf; i++)
        for (const DChain &h : F[i]->chain)
            if (h.ntask > 0 && k < 6) e[k++] = h.ctrl.p + 2;
    hipLaunchKernelGGL(solve_status_kernel, dim3(1), dim3(1), 0, c.stream, out, host_code, e[0], e[1], e[2], e[3], e[4],
                       e[5], chain_code);
    CPK_HIP(hipGetLastError());
}
// test hook (engine option fail_inject "R:chain:K"): set a chain's device error word, as a wait
// that timed out would; false if the factor has no chain
bool debug_set_chain_error(Ctx &c, const DFactor &F) {
    for (const DChain &h : F.chain)
        if (h.ntask > 0) {
            const uint32_t one = 1;
            CPK_HIP(hipMemcpyAsync(h.ctrl.p + 2, &one, sizeof one, hipMemcpyHostToDevice, c.stream));
            CPK_HIP(hipStreamSynchronize(c.stream));
            return true;
        }
    return false;
}

// the block kernel a chain runs: 256 threads (blocks of <= 512 rows / 3072 entries, the single-
// GPU default) or 512 (<= 1024 / 4096, the distributed default); 0: none
static int chain_tpb(const DFactor &d) {
    if (d.sweep_threads[1] == 256 && d.sweep_rows[1] <= 512 && d.sweep_cap[1] <= 3072) return 256;
    if (d.sweep_threads[1] == 512 && d.sweep_rows[1] <= 1024 && d.sweep_cap[1] <= 4096) return 512;
    return 0;
}

static void build_chain_kind(DFactor &d, int kind, const std::vector<int32_t> &blk, const std::vector<int32_t> &meta,
                             const std::vector<uint32_t> &fptr, const std::vector<int32_t> &fcol,
                             const std::vector<uint32_t> &bptr, const std::vector<int32_t> &bcol) {
    DChain &ch = d.chain[kind];
    const int64_t R = (int64_t)d.round_ptr.size() - 1;
    const int64_t b1 = d.round_ptr[d.chain_first], be = d.round_ptr[R];
    const int64_t N = d.N, base = meta[(size_t)b1 * 8];  // the chain's first row
    // forward tasks for blocks [b1, bf), the last round's blocks [bf, be) as last tasks (full
    // chain), backward tasks for blocks [b1, bb) from the highest round down
    const int64_t bl = d.round_ptr[R - 1];
    const int64_t bf = kind == kChainFull ? bl : (kind == kChainFwd ? be : b1);
    const int64_t nlast = kind == kChainFull ? be - bl : 0;
    const int64_t bb = kind == kChainFull ? bl : (kind == kChainBwd ? be : b1);
    const int64_t nfl = (bf - b1) + nlast, nt = nfl + (bb - b1);
    if (nt <= 0 || nt >= (1 << 28)) return;
    auto fwd_task = [&](int64_t b) { return (int32_t)(b - b1); };  // forward and last tasks: block order
    auto bwd_task = [&](int64_t b) {
        return (kind == kChainFull && b >= bl) ? (int32_t)(b - b1) : (int32_t)(nfl + (bb - 1 - b));
    };
    std::vector<int32_t> task((size_t)nt), dptr((size_t)nt + 1, 0), didx, deps;
    bool ok = true;
    auto emit = [&](int32_t t) {
        std::sort(deps.begin(), deps.end());
        deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
        for (int32_t p : deps) ok = ok && p >= 0 && p < t;
        didx.insert(didx.end(), deps.begin(), deps.end());
        dptr[(size_t)t + 1] = (int32_t)didx.size();
        deps.clear();
    };
    auto upper = [&](int32_t c) { return c >= base && c < N; };  // a row of this launch (T rows: c >= N)
    for (int64_t b = b1; b < b1 + nfl && ok; b++) {  // forward / last
        const int32_t *m = &meta[(size_t)b * 8];
        const bool last = b >= bf;
        for (int32_t i = m[0]; i < m[1]; i++) {
            for (uint32_t e = fptr[i]; e < fptr[i + 1]; e++)
                if (upper(fcol[e]) && (fcol[e] < m[0] || fcol[e] >= m[1])) deps.push_back(fwd_task(blk[(size_t)(fcol[e] - base)]));
            if (last)  // a last-round block's backward terms must stay inside it (sptrsv_last_kernel)
                for (uint32_t e = bptr[i]; e < bptr[i + 1]; e++)
                    if (upper(bcol[e]) && (bcol[e] < m[0] || bcol[e] >= m[1])) ok = false;
        }
        task[(size_t)fwd_task(b)] = (int32_t)((last ? 1 : 0) << 28 | b);
        emit(fwd_task(b));
    }
    for (int64_t b = bb - 1; b >= b1 && ok; b--) {  // backward, highest round first
        const int32_t *m = &meta[(size_t)b * 8];
        if (kind == kChainFull) deps.push_back(fwd_task(b));  // its own forward values, this launch
        for (int32_t i = m[0]; i < m[1]; i++)
            for (uint32_t e = bptr[i]; e < bptr[i + 1]; e++)
                if (upper(bcol[e]) && (bcol[e] < m[0] || bcol[e] >= m[1])) deps.push_back(bwd_task(blk[(size_t)(bcol[e] - base)]));
        task[(size_t)bwd_task(b)] = (int32_t)(2 << 28 | b);
        emit(bwd_task(b));
    }
    if (!ok) return;
    ch.task.upload(task);
    ch.dptr.upload(dptr);
    ch.didx.upload(didx.empty() ? std::vector<int32_t>{0} : didx);
    ch.flag.alloc((size_t)nt);
    CPK_HIP(hipMemset(ch.flag.p, 0, ch.flag.bytes()));
    ch.ctrl.alloc(4);
    CPK_HIP(hipMemset(ch.ctrl.p, 0, ch.ctrl.bytes()));
    ch.tpb = chain_tpb(d);
    ch.ntask = nt;
}

static void build_chain(DFactor &d, const std::vector<int32_t> &meta, const std::vector<uint32_t> &fptr,
                        const std::vector<int32_t> &fcol, const std::vector<uint32_t> &bptr,
                        const std::vector<int32_t> &bcol) {
    for (DChain &c : d.chain) c.ntask = 0;
    const int64_t R = (int64_t)d.round_ptr.size() - 1;
    if (d.no_chain || d.no_upper || R < 3 || !chain_tpb(d)) return;
    // the chained rounds: the narrow top [first, R), two rounds at least, every one through the
    // block kernel
    int64_t first = R;
    while (first > 1 && d.round_ptr[first] - d.round_ptr[first - 1] <= d.chain_wide) first--;
    if (R - first < 2) return;
    for (int64_t r = first; r < R; r++)
        if (r >= (int64_t)d.round_fits.size() || !d.round_fits[r]) return;
    d.chain_first = first;
    const int64_t N = d.N, base = meta[(size_t)d.round_ptr[first] * 8];
    std::vector<int32_t> blk((size_t)(N - base), -1);
    for (int64_t b = d.round_ptr[first]; b < d.round_ptr[R]; b++)
        for (int32_t i = meta[(size_t)b * 8]; i < meta[(size_t)b * 8 + 1]; i++) blk[(size_t)(i - base)] = (int32_t)b;
    for (int32_t x : blk)
        if (x < 0) return;  // upper rows not all in upper blocks
    for (int k : {kChainFull, kChainFwd, kChainBwd}) build_chain_kind(d, k, blk, meta, fptr, fcol, bptr, bcol);
}

static bool chain_ok(const DFactor &F, int kind) {
    return F.chain[kind].ntask > 0 && !F.no_chain && (kind != kChainFull || fuse_last_ok(F));
}

template <int TPB, int RPU, int EPU>
static void launch_chain_t(Ctx &c, const DFactor &F, int kind, const FwdIn &in, double *w, double *out, bool add,
                           const int *run, const int *active, double *ys, const PackArgs &pk) {
    const DChain &h = F.chain[kind];
    const size_t lds = std::max<size_t>(sweep_lds_bytes(RPU * TPB, EPU * TPB), (size_t)CPK_CHAIN_LDS_MIN);
    static const bool lds_ok = lds <= 64 * 1024 ||
        (hipFuncSetAttribute((const void *)sptrsv_chain_kernel<TPB, RPU, EPU, false>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess &&
         hipFuncSetAttribute((const void *)sptrsv_chain_kernel<TPB, RPU, EPU, true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess);
    if (!lds_ok) throw Error(CPK_ERR_HIP, "sptrsv_chain_kernel: LDS image not admitted");
    const Img img{RPU * TPB, EPU * TPB};  // narrow rounds: every task resident at the kernel's image
    const BlkMeta *meta = reinterpret_cast<const BlkMeta *>(F.meta.p);
    const size_t ldsb = std::max<size_t>(img_bytes(img), (size_t)CPK_CHAIN_LDS_MIN);
    const ChainArgs ch{h.task.p, h.dptr.p, h.didx.p, h.flag.p, h.ctrl.p, (int)h.ntask};
    if (add)
        hipLaunchKernelGGL((sptrsv_chain_kernel<TPB, RPU, EPU, true>), dim3((unsigned)h.ntask), dim3(TPB), ldsb, c.stream,
                           ch, meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p,
                           F.perm.p, in.xin, in.neg_from, in.sched_in, in.xs, w, out, run, active, ys, pk, ufold_of(F), img);
    else
        hipLaunchKernelGGL((sptrsv_chain_kernel<TPB, RPU, EPU, false>), dim3((unsigned)h.ntask), dim3(TPB), ldsb,
                           c.stream, ch, meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.bptr.p, F.bcol.p, F.bval.p,
                           F.D.p, F.perm.p, in.xin, in.neg_from, in.sched_in, in.xs, w, out, run, active, ys, pk, ufold_of(F), img);
    CPK_HIP(hipGetLastError());
}
static void launch_chain(Ctx &c, const DFactor &F, int kind, const FwdIn &in, double *w, double *out, bool add,
                         const int *run, const int *active, double *ys, const PackArgs &pk) {
    if (F.chain[kind].tpb == 512) launch_chain_t<512, 2, 8>(c, F, kind, in, w, out, add, run, active, ys, pk);
    else launch_chain_t<256, 2, 12>(c, F, kind, in, w, out, add, run, active, ys, pk);
}

void check_chain(const DFactor &F) {
    for (const DChain &h : F.chain) {
        if (h.ntask <= 0) continue;
        uint32_t err = 0;
        CPK_HIP(hipMemcpy(&err, h.ctrl.p + 2, sizeof err, hipMemcpyDeviceToHost));
        if (err) {
            CPK_HIP(hipMemset(h.ctrl.p + 2, 0, sizeof err));
            throw Error(CPK_ERR_HIP, "sweep chain: a block's wait for its producers timed out");
        }
    }
}

template <int TPB, int RPU, int EPU>
static bool upper_round_t(Ctx &c, const DFactor &F, int64_t r, bool bwd, bool add, const double *xin,
                          int64_t neg_from, double *w, double *out, const int *run, const int *active, int sched_in,
                          double *ys, double *xs, const PackArgs &pk) {
    if (F.sweep_threads[1] != TPB || F.sweep_rows[1] > RPU * TPB || F.sweep_cap[1] > EPU * TPB ||
        r >= (int64_t)F.round_fits.size() || !F.round_fits[r])
        return false;
    const int64_t b0 = F.round_ptr[r], nb = F.round_ptr[r + 1] - b0;
    if (!nb) return true;
    const size_t lds = sweep_lds_bytes(RPU * TPB, EPU * TPB);  // the kernel's image (>= the configured block)
    static const bool lds_ok = lds <= 64 * 1024 ||
        (hipFuncSetAttribute((const void *)sptrsv_upper_kernel<TPB, RPU, EPU, false, false>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess &&
         hipFuncSetAttribute((const void *)sptrsv_upper_kernel<TPB, RPU, EPU, true, true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess &&
         hipFuncSetAttribute((const void *)sptrsv_upper_kernel<TPB, RPU, EPU, true, false>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess);
    if (!lds_ok) return false;
    const BlkMeta *meta = reinterpret_cast<const BlkMeta *>(F.meta.p);
    // the round's own image only where it raises residency for a round that needs it: a round of
    // at most (kernel-image blocks per CU) x CUs workgroups is resident at once already, and a
    // smaller image would let some CUs take more of its blocks than others (S10's first upper
    // round, 1024 blocks: 4 per CU on every CU, or 5 on some and 3 on others)
    static const int64_t resident = [] {
        int cus = 256, dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return (int64_t)cus * (int64_t)std::max<size_t>(1, (160 * 1024) / sweep_lds_bytes(RPU * TPB, EPU * TPB));
    }();
    const Img img = nb > resident ? launch_img(F, b0, b0 + nb, RPU * TPB, EPU * TPB) : Img{RPU * TPB, EPU * TPB};
    const size_t ldsr = img_bytes(img);
    if (!bwd)
        hipLaunchKernelGGL((sptrsv_upper_kernel<TPB, RPU, EPU, false, false>), dim3((unsigned)nb), dim3(TPB), ldsr,
                           c.stream, b0, meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.D.p, F.perm.p, xin,
                           neg_from, w, out, run, active, sched_in, ys, xs, pk, ufold_of(F), img);
    else if (add)
        hipLaunchKernelGGL((sptrsv_upper_kernel<TPB, RPU, EPU, true, true>), dim3((unsigned)nb), dim3(TPB), ldsr,
                           c.stream, b0, meta, F.lvl_row.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p, F.perm.p, xin,
                           neg_from, w, out, run, active, sched_in, ys, xs, pk, ufold_of(F), img);
    else
        hipLaunchKernelGGL((sptrsv_upper_kernel<TPB, RPU, EPU, true, false>), dim3((unsigned)nb), dim3(TPB), ldsr,
                           c.stream, b0, meta, F.lvl_row.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p, F.perm.p, xin,
                           neg_from, w, out, run, active, sched_in, ys, xs, pk, ufold_of(F), img);
    return true;
}

// upper round r through sptrsv_upper_kernel when the configuration matches the instantiation
// (512 threads: blocks of <= 1024 rows / 4096 entries).  Measured at S10 and not kept: 1024
// threads with blocks of 1536 / 6144 and 2048 / 8192 (still 4 rounds; sweeps 2-7 % slower).
static bool upper_round(Ctx &c, const DFactor &F, int64_t r, bool bwd, bool add, const double *xin,
                        int64_t neg_from, double *w, double *out, const int *run, const int *active, int sched_in,
                        double *ys, double *xs, const PackArgs &pk) {
    if (F.no_upper) return false;
    // 256 threads (blocks of <= 512 rows / 3072 entries, a 38 KB image): four blocks per CU, for a
    // schedule whose first upper round has more blocks than 512-thread images keep resident
    return upper_round_t<512, 2, 8>(c, F, r, bwd, add, xin, neg_from, w, out, run, active, sched_in, ys, xs, pk) ||
           upper_round_t<256, 2, 12>(c, F, r, bwd, add, xin, neg_from, w, out, run, active, sched_in, ys, xs, pk);
}

// SPLIT > 1: the workgroup is one wave holding SPLIT independent logical blocks of TPB lanes
// (TPB * SPLIT = 64), each with its own LDS image.  A level that occupies a few rows then costs
// one instruction stream for SPLIT blocks instead of one per block; lanes of different logical
// blocks never synchronise (within a single wave __syncthreads is a no-op fence).
#ifdef CPK_PIPE_STAMPS
// diagnostic build only (make HIPEXTRA=-DCPK_PIPE_STAMPS): per-workgroup start / end of the last
// round-0 launch (s_memrealtime, 100 MHz), read by cpk_debug_pipe_stamps (tools/pipe_stamps.py)
__device__ uint64_t g_pipe_stamps[2 * 16384];
#endif
template <int TPB, int RPT, int EPT, bool BWD, bool ADD, int SPLIT = 1, bool LOC = false, bool RES = false>
#ifndef CPK_PIPE_WAVES
#define CPK_PIPE_WAVES 4  // waves per SIMD the round-0 kernel's registers allow (4: 128 VGPRs)
#endif
__global__ __launch_bounds__(TPB * SPLIT) __attribute__((amdgpu_waves_per_eu(SPLIT == 1 ? CPK_PIPE_WAVES : 1))) void sptrsv_pipe_kernel(
    int64_t blk0, int64_t nblk, const BlkMeta *__restrict__ meta, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ D, const int32_t *__restrict__ perm, const double *__restrict__ xin,
    int64_t neg_from, double *w, double *out, const int *run, const int *active, int sched_in, double *ys,
    int skip0, double *xs, const int16_t *__restrict__ col16, ResArgs ra, const BlkMeta *__restrict__ ameta,
    const int32_t *__restrict__ aptr, PackArgs pk) {
    static_assert(SPLIT == 1 || TPB * SPLIT == 64, "split blocks must share one wave");
    static_assert(!LOC || !BWD, "block-local columns: forward round 0 only");
    static_assert(!RES || (LOC && SPLIT == 1), "fused residual: forward round 0 with block-local columns");
    // sched_in: forward, the input is in schedule order; backward, w is dead after the sweep
    // (launch_sptrsv_bwd's wdead).  perm is read for the forward gather (unless the input is in
    // schedule order) and for the backward scatter (unless the solution stays in schedule order)
    const bool need_perm = BWD ? out != nullptr : !sched_in;
    constexpr int R = RPT * TPB, CAP = EPT * TPB;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (skip(run, active)) return;
    if (!BWD) pack_inputs(pk, (int64_t)blockIdx.x * (TPB * SPLIT) + threadIdx.x);  // rank 0's T inputs, piggyback
    const int sub = SPLIT > 1 ? (int)threadIdx.x / TPB : 0;
    SweepLds S(smem + (SPLIT > 1 ? sub * (int)sweep_lds_bytes_dev(R, CAP) : 0), R, CAP);
    const int tid = SPLIT > 1 ? (int)threadIdx.x % TPB : (int)threadIdx.x;
    const int64_t G = (int64_t)gridDim.x * SPLIT;
    // prefetched registers of the next block
    uint32_t q[RPT];
    int32_t sp[RPT], lvr[RPT];
    double wr[RPT], dr[RPT];
    int32_t cc[EPT];
    double vv[EPT];
    // RES: the block's Kps entry range, its rows' Kps pointers and xs, and the first chunk of
    // Kps entries (CAP of them)
    uint32_t kb0 = 0, kb1 = 0;
    int32_t kc[RES ? EPT : 1];  // columns only: the values load beside the y gathers
    auto issue = [&](const BlkMeta &m) {
        const int nr = m.r1 - m.r0, nl = (m.l1 & kMetaL1Mask) - m.l0;
        const uint32_t e0 = BWD ? (uint32_t)m.be0 : (uint32_t)m.fe0;
        const int ne = BWD ? m.be1 - m.be0 : m.fe1 - m.fe0;
        if (RES) {
            kb0 = ra.ptr[m.r0], kb1 = ra.ptr[m.r1];
#pragma unroll
            for (int j = 0; j < (RES ? EPT : 0); j++) {
                const uint32_t e = kb0 + (uint32_t)(tid + j * TPB);
                if (e < kb1) kc[j] = __builtin_nontemporal_load(ra.col + e);
            }
        }
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const int i = tid + j * TPB;
            const int rr = m.r0 + (i < nr ? i : nr - 1);  // clamped: later gathers need no predicate
            // the row arrays are streamed once per sweep too
            q[j] = __builtin_nontemporal_load(ptr + rr);
            sp[j] = need_perm ? __builtin_nontemporal_load(perm + rr) : rr;
            if (BWD) wr[j] = w[rr], dr[j] = __builtin_nontemporal_load(D + rr);
            if (i < nl) lvr[j] = __builtin_nontemporal_load(lvl_row + m.l0 + i);
        }
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const int e = tid + j * TPB;
            if (e < ne) {  // streamed once per sweep: non-temporal, keeps L2 for the gathered vector
                if (LOC) cc[j] = __builtin_nontemporal_load(col16 + e0 + e);
                else cc[j] = __builtin_nontemporal_load(col + e0 + e);
                vv[j] = __builtin_nontemporal_load(val + e0 + e);
            }
        }
    };
#ifdef CPK_PIPE_STAMPS
    const uint64_t t_start = (uint64_t)wall_clock64();
    struct Stamp {
        uint64_t t0;
        __device__ ~Stamp() {
            if (threadIdx.x == 0 && blockIdx.x < 16384)
                g_pipe_stamps[2 * blockIdx.x] = t0, g_pipe_stamps[2 * blockIdx.x + 1] = (uint64_t)wall_clock64();
        }
    } stamp{t_start};
#endif
    // the blocks of this workgroup: the host's assignment (aptr: ameta[aptr[g] .. aptr[g + 1]),
    // balanced by cost, DFactor::plan_round0) or, without one, every G-th block from blk0 + g
    const bool asg = aptr != nullptr;
    int64_t b = asg ? (int64_t)aptr[blockIdx.x] : blk0 + (int64_t)blockIdx.x * SPLIT + sub;
    const int64_t bend = asg ? (int64_t)aptr[blockIdx.x + 1] : blk0 + nblk;
    const int64_t bstep = asg ? 1 : G;
    const BlkMeta *const msrc = asg ? ameta : meta;
    auto tail = [&]() {
        for (int64_t k = ra.tail0 + (int64_t)blockIdx.x * TPB + tid; k < ra.tail1; k += (int64_t)gridDim.x * TPB) {
            const uint32_t ka = ra.ptr[k], kz = ra.ptr[k + 1];
            double acc = 0.0;
            for (uint32_t e = ka; e < kz; e++) {
                const double p = ra.val[e] * ra.y[ra.col[e]];
                acc += p;
            }
            w[k] = ra.xs[k] - acc;
        }
    };
    if (b >= bend) {
        if (RES) tail();
        return;
    }
    BlkMeta cur = msrc[b];
    issue(cur);
    while (true) {
#ifdef CPK_PIPE_STAMPS
        const uint64_t tb = (uint64_t)clock64();
#endif
        const int nr = cur.r1 - cur.r0, nl = (cur.l1 & kMetaL1Mask) - cur.l0;
        const uint32_t e0 = BWD ? (uint32_t)cur.be0 : (uint32_t)cur.fe0;
        const int ne = BWD ? cur.be1 - cur.be0 : cur.fe1 - cur.fe0;
        const int r0 = cur.r0, r1 = cur.r1;
        // registers -> LDS, with the dependent gathers (all in flight at once: forward the input
        // through perm, backward-accumulate the output rows read back after the levels)
        double xg[RPT];
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const int i = tid + j * TPB;
            if (!BWD && !RES) xg[j] = xin[sp[j]];
            if (BWD && ADD) xg[j] = ys ? ys[r0 + (i < nr ? i : nr - 1)] : out[sp[j]];
        }
        if (RES) {  // r = xs - Kps*y for the block's rows, through the (free) value region of LDS
            // the L columns go to LDS first (their region is not used here): fewer live registers
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                const int e = tid + j * TPB;
                if (e < ne) S.c[e] = (int16_t)cc[j];
            }
#pragma unroll
            for (int j = 0; j < RPT; j++) {  // likewise the row pointers and level bounds
                const int i = tid + j * TPB;
                if (i < nr) S.p[i] = (int16_t)(q[j] - e0);
                if (i < nl) S.lv[i] = (int16_t)(lvr[j] - r0);
            }
            // the rows' Kps pointers and xs load beside the first chunk's gathers (not prefetched
            // with the block: the level phase holds the next block's registers)
            uint32_t kqa[RPT], kqb[RPT];
            double xsr[RPT], acc[RPT];
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                const int i = tid + j * TPB, rr = r0 + (i < nr ? i : nr - 1);
                kqa[j] = ra.ptr[rr], kqb[j] = ra.ptr[rr + 1], xsr[j] = ra.xs[rr];
                acc[j] = 0.0;
            }
            for (uint32_t c0 = kb0;; c0 += (uint32_t)CAP) {
                if (c0 != kb0) {  // a block with more than CAP Kps entries: the next chunk
#pragma unroll
                    for (int j = 0; j < (RES ? EPT : 0); j++) {
                        const uint32_t e = c0 + (uint32_t)(tid + j * TPB);
                        if (e < kb1) kc[j] = __builtin_nontemporal_load(ra.col + e);
                    }
                }
                // two halves, the second issued after the first is in LDS: half the registers
                constexpr int H = (EPT + 1) / 2;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    double kv[H], yg[H];
#pragma unroll
                    for (int u = 0; u < H; u++) {
                        const int j = h * H + u;
                        const uint32_t e = c0 + (uint32_t)(tid + j * TPB);
                        if (j < EPT) {
                            kv[u] = __builtin_nontemporal_load(ra.val + (e < kb1 ? e : 0));  // clamped: a valid entry
                            yg[u] = ra.y[e < kb1 ? kc[j] : 0];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < H; u++) {
                        const int j = h * H + u;
                        const uint32_t e = c0 + (uint32_t)(tid + j * TPB);
                        if (j < EPT && e < kb1) S.v[e - c0] = kv[u] * yg[u];
                    }
                    if (h == 0) asm volatile("" ::: "memory");
                }
                __syncthreads();
                const uint32_t c1 = c0 + (uint32_t)CAP;
#pragma unroll
                for (int j = 0; j < RPT; j++) {
                    if (tid + j * TPB < nr) {
                        const uint32_t lo = kqa[j] > c0 ? kqa[j] : c0, hi = kqb[j] < c1 ? kqb[j] : c1;
                        for (uint32_t e = lo; e < hi; e++) acc[j] += S.v[e - c0];
                    }
                }
                __syncthreads();
                if (kb1 <= c1) break;
            }
#pragma unroll
            for (int j = 0; j < RPT; j++) xg[j] = xsr[j] - acc[j];
        }
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const int i = tid + j * TPB;
            if (i < nr) {
                if (!RES) S.p[i] = (int16_t)(q[j] - e0);
                if (BWD) S.w[i] = wr[j] / dr[j];
                else S.w[i] = (sp[j] >= neg_from) ? -xg[j] : xg[j];
                if (!BWD && xs) xs[r0 + i] = S.w[i];  // the input in schedule order, for the residual
            }
            if (!RES && i < nl) S.lv[i] = (int16_t)(lvr[j] - r0);
        }
        int32_t dst[RPT];
#pragma unroll
        for (int j = 0; j < RPT; j++) dst[j] = sp[j];
        if (tid == 0) S.p[nr] = (int16_t)ne, S.lv[nl] = (int16_t)nr, S.w[R] = 1.0;
        if (tid < kSweepPad) S.c[ne + tid] = (int16_t)R;
        double g[EPT];  // backward: w of the rows of earlier launches, every gather in flight at once
        if (BWD) {
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                const int e = tid + j * TPB;
                const bool out = e < ne && (cc[j] < r0 || cc[j] >= r1);
                g[j] = w[out ? cc[j] : r0];
            }
        }
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const int e = tid + j * TPB;
            if (e < ne) {
                if (LOC) {  // already block-local (fcol16)
                    if (!RES) S.c[e] = (int16_t)cc[j];
                    S.v[e] = vv[j];
                } else {
                    const int32_t c = cc[j];
                    const bool local = c >= r0 && c < r1;
                    S.c[e] = local ? (int16_t)(c - r0) : (int16_t)R;
                    S.v[e] = local ? vv[j] : vv[j] * (BWD ? g[j] : w[c]);
                }
            }
        }
        __syncthreads();
        const int64_t bn = b + bstep;
        BlkMeta nxt;
        if (bn < bend) {
            nxt = msrc[bn];
            issue(nxt);  // in flight during the level phase
        }
        // skip0: level 0 holds only rows without entries (the G pivots are in the blocks)
        // lane-owned rows for the backward sweep only: A/B at S10 (profiles/r03_level_ab_v2.txt),
        // backward 193.9 -> 186.7 us, but forward 211 -> 232 us and the fused forward 270 -> 286
        if (CPK_R0_DATAFLOW && (CPK_R0_DATAFLOW == 1 || !BWD) && SPLIT == 1 && TPB == kWave)
            levels_dataflow<BWD, BWD ? CPK_R0_DF_CH_BWD : CPK_R0_DF_CH_FWD, false, R / kWave>(S, nr, R, ne, tid);
        else if (CPK_LEVEL_OWN && SPLIT == 1 && BWD) levels_owned<TPB, RPT, BWD, CPK_PIPE_CH>(S, nl, nr, skip0 != 0, tid);
        else if (CPK_LEVEL_GROUP && SPLIT == 1 && TPB == kWave && !BWD) levels_grouped_fwd<CPK_PIPE_CH>(S, nl, skip0 != 0, tid);
        else sweep_levels<TPB, BWD, false, CPK_PIPE_CH, false, true>(S, nl, skip0 != 0, tid);
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const int i = tid + j * TPB;
            if (i < nr) {
                const double z = S.w[i];
                // round 0 is the backward sweep's last round; the caller says when nothing reads
                // its w afterwards (backward: sched_in carries launch_sptrsv_bwd's wdead)
                if (!BWD || !sched_in) w[r0 + i] = z;
                if (BWD) {
                    if (out) {
                        const double o = ADD ? xg[j] + z : z;
                        out[dst[j]] = o;
                        pack_put(pk, dst[j], o);
                    } else {  // the solution stays in schedule order: packed by schedule row
                        const double o = ADD ? xg[j] + z : z;
                        if (ADD) ys[r0 + i] = o;
                        pack_put(pk, r0 + i, o);
                    }
                } else {
                    pack_put(pk, r0 + i, z);
                }
            }
        }
#ifdef CPK_PIPE_STAMPS
        if (SPLIT == 1 && tid == 0 && cur.l0 < kBlkCycMax)  // keyed by l0: valid under the assignment too
            g_blk_cyc[(BWD ? (ADD ? 3 : 2) : (RES ? 1 : 0)) * kBlkCycMax + cur.l0] = (uint64_t)clock64() - tb;
#endif
        if (bn >= bend) break;
        __syncthreads();
        b = bn;
        cur = nxt;
    }
    if (RES) tail();
}

// threads == 32 in a sweep configuration selects the split kernel: 2 logical blocks of 32 lanes
// per 64-lane wave
template <int TPB, int RPT, int EPT, int SPLIT = 1>
static bool pipe_round(Ctx &c, const DFactor &F, bool bwd, bool add, const double *xin, int64_t neg_from,
                       double *w, double *out, const int *run, const int *active, int sched_in, double *ys,
                       double *xs, const ResArgs *ra = nullptr, int64_t *plan_grid = nullptr, const PackArgs *pk = nullptr,
                       bool *pk_used = nullptr) {
    if (F.sweep_threads[0] != TPB || F.sweep_rows[0] != RPT * TPB || F.sweep_cap[0] != EPT * TPB) return false;
    if (ra && (bwd || F.fcol16.n == 0 || SPLIT != 1)) return false;  // fused residual: one instantiation
    const int64_t nb = F.round_ptr[1] - F.round_ptr[0];
    const size_t lds = sweep_lds_bytes(RPT * TPB, EPT * TPB) * SPLIT;
    int occ = 0;
    const bool loc = !bwd && F.fcol16.n > 0;
    constexpr bool kRes = SPLIT == 1;  // the fused residual kernel exists for unsplit blocks only
    const void *fn = ra ? (const void *)sptrsv_pipe_kernel<TPB, RPT, EPT, false, false, SPLIT, true, kRes>
                  : bwd ? (add ? (const void *)sptrsv_pipe_kernel<TPB, RPT, EPT, true, true, SPLIT>
                                : (const void *)sptrsv_pipe_kernel<TPB, RPT, EPT, true, false, SPLIT>)
                         : loc ? (const void *)sptrsv_pipe_kernel<TPB, RPT, EPT, false, false, SPLIT, true>
                               : (const void *)sptrsv_pipe_kernel<TPB, RPT, EPT, false, false, SPLIT>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, TPB * SPLIT, lds) != hipSuccess || occ < 1) occ = 1;
    // at most CPK_PIPE_WAVES waves per SIMD, even when a variant's registers would allow more: the
    // assignment's dispatch-slot speeds (plan_round0) are measured at four, and a fifth wave on
    // some SIMDs only (the LDS caps a CU at 18 workgroups) made the forward sweep 15 % slower
    // (a 96-VGPR build, r04o)
    occ = std::min(occ, std::max(1, CPK_PIPE_WAVES * 4 * kWave / (TPB * SPLIT)));
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>((nb + SPLIT - 1) / SPLIT, (int64_t)occ * cus));
    // the forward pack puts one T input per thread of the grid: only when the grid covers them
    if (pk && !bwd && (int64_t)pk->ntdof > grid * TPB * SPLIT) pk = nullptr;
    if (pk_used) *pk_used = pk != nullptr;
    if (plan_grid) {  // plan_round0: the grid this launch would use (no assignment for split blocks)
        *plan_grid = SPLIT == 1 ? grid : 0;
        return true;
    }
    const BlkMeta *meta = reinterpret_cast<const BlkMeta *>(F.meta.p);
    const dim3 blk(TPB * SPLIT);
    // the host's balanced assignment of this variant, when it was made for this grid
    const int v = ra ? 1 : (bwd ? 2 : 0);
    const bool use_asg = SPLIT == 1 && F.agrid[v] == grid && F.aptr[v].n == (size_t)grid + 1;
    const BlkMeta *am = use_asg ? reinterpret_cast<const BlkMeta *>(F.ameta[v].p) : nullptr;
    const int32_t *ap = use_asg ? F.aptr[v].p : nullptr;
    if (ra)
        hipLaunchKernelGGL((sptrsv_pipe_kernel<TPB, RPT, EPT, false, false, SPLIT, true, kRes>), dim3((unsigned)grid),
                           blk, lds, c.stream, F.round_ptr[0], nb, meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p,
                           F.D.p, F.perm.p, xin, neg_from, w, out, run, active, 1, ys, F.skip0 ? 1 : 0, xs,
                           (const int16_t *)F.fcol16.p, *ra, am, ap, pk ? *pk : PackArgs{});
    else if (loc)
        hipLaunchKernelGGL((sptrsv_pipe_kernel<TPB, RPT, EPT, false, false, SPLIT, true>), dim3((unsigned)grid), blk,
                           lds, c.stream, F.round_ptr[0], nb, meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.D.p,
                           F.perm.p, xin, neg_from, w, out, run, active, sched_in, ys, F.skip0 ? 1 : 0, xs,
                           (const int16_t *)F.fcol16.p, ResArgs{}, am, ap, pk ? *pk : PackArgs{});
    else if (!bwd)
        hipLaunchKernelGGL((sptrsv_pipe_kernel<TPB, RPT, EPT, false, false, SPLIT>), dim3((unsigned)grid), blk, lds,
                           c.stream, F.round_ptr[0], nb, meta, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.D.p,
                           F.perm.p, xin, neg_from, w, out, run, active, sched_in, ys, F.skip0 ? 1 : 0, xs,
                           (const int16_t *)nullptr, ResArgs{}, am, ap, pk ? *pk : PackArgs{});
    else if (add)
        hipLaunchKernelGGL((sptrsv_pipe_kernel<TPB, RPT, EPT, true, true, SPLIT>), dim3((unsigned)grid), blk, lds,
                           c.stream, F.round_ptr[0], nb, meta, F.lvl_row.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p,
                           F.perm.p, xin, neg_from, w, out, run, active, sched_in, ys, F.skip0 ? 1 : 0, xs,
                           (const int16_t *)nullptr, ResArgs{}, am, ap, pk ? *pk : PackArgs{});
    else
        hipLaunchKernelGGL((sptrsv_pipe_kernel<TPB, RPT, EPT, true, false, SPLIT>), dim3((unsigned)grid), blk, lds,
                           c.stream, F.round_ptr[0], nb, meta, F.lvl_row.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p,
                           F.perm.p, xin, neg_from, w, out, run, active, sched_in, ys, F.skip0 ? 1 : 0, xs,
                           (const int16_t *)nullptr, ResArgs{}, am, ap, pk ? *pk : PackArgs{});
    return true;
}

// round 0 through the pipelined kernel when its configuration is one of the instantiated ones
// (plan_grid: nothing is launched, the grid of the matching instantiation is returned)
static bool pipe_round0(Ctx &c, const DFactor &F, bool bwd, bool add, const double *xin, int64_t neg_from,
                        double *w, double *out, const int *run, const int *active, int sched_in, double *ys,
                        double *xs, int64_t *plan_grid = nullptr, const PackArgs *pk = nullptr, bool *pk_used = nullptr) {
    if (!F.pipelined || F.round_ptr.size() < 2) return false;
#define CPK_PR(...) pipe_round<__VA_ARGS__>(c, F, bwd, add, xin, neg_from, w, out, run, active, sched_in, ys, xs, nullptr, plan_grid, pk, pk_used)
    return CPK_PR(32, 6, 18, 2) || CPK_PR(32, 4, 12, 2) || CPK_PR(32, 8, 24, 2) || CPK_PR(128, 2, 6) ||
           CPK_PR(64, 3, 9) || CPK_PR(64, 4, 12) || CPK_PR(64, 6, 18) || CPK_PR(64, 8, 24) || CPK_PR(128, 1, 4) ||
           CPK_PR(256, 1, 3);
#undef CPK_PR
}

// the fused-residual round-0 instantiations (launch_sptrsv_fwd_resid)
static bool pipe_round0_resid(Ctx &c, const DFactor &F, double *r, const int *run, const ResArgs &ra,
                              int64_t *plan_grid = nullptr, const PackArgs *pk = nullptr, bool *pk_used = nullptr) {
#define CPK_PR(...) pipe_round<__VA_ARGS__>(c, F, false, false, r, INT64_MAX, r, nullptr, run, nullptr, 1, nullptr, nullptr, &ra, plan_grid, pk, pk_used)
    return CPK_PR(64, 3, 9) || CPK_PR(64, 4, 12) || CPK_PR(128, 2, 6) || CPK_PR(64, 6, 18);
#undef CPK_PR
}

// ---- round-0 block assignment (longest processing time first) ---------------------------------
// A persistent round-0 workgroup used to take every G-th block, so the launch ended with the
// workgroup whose fixed share happened to cost most: 9-13 % of each launch was tail (DESIGN.md
// 7a, per-workgroup stamps).  Block costs are static, so the host assigns the blocks to the
// launch's G workgroups once: blocks by descending modelled cost, each to the least loaded
// workgroup so far; a workgroup then walks its blocks in ascending order.  The arithmetic of
// every block is unchanged (bit-identical), only which workgroup runs it and when.
// Cost model: c0 + c1 levels + c2 rows + c3 entries (+ c4 Kps entries) per block and variant.
static const double kR0Cost[3][5] = {
    // The s_memtime stamps (tools/blk_cycles.py, profiles/r03_blk_cycles_v0.log) fit poorly per
    // block (R^2 0.1-0.6: a block's time depends on what shares its CU), but the level count
    // dominates every fit (~1500-1900 cycles per level) and, replayed on the measured cycles,
    // LPT by levels alone gave the lowest maximum: 1.07-1.12 x the median workgroup against
    // 1.12-1.18 for the stride.  Rows break ties.
    {0.0, 1.0, 1e-3, 0.0, 0.0},  // forward
    {0.0, 1.0, 1e-3, 0.0, 0.0},  // forward with the fused refinement residual
    {0.0, 1.0, 1e-3, 0.0, 0.0},  // backward
};

// Relative speed of the workgroups of each dispatch slot: with four workgroups on every SIMD,
// the first dispatched on each SIMD (blockIdx < 4 x CUs) runs fastest and the fourth slowest --
// the SIMD issues older waves first.  Per-workgroup stamps at S10 with equal modelled work per
// workgroup (profiles/r03_stamps_v2.log): forward 210 / 213 / 221 / 230 us, backward 139 / 148 /
// 157 / 166 us by slot, whatever the XCD (means per XCD within 1 %).  Work is assigned in
// proportion; with those speeds the slots finished at 202 / 206 / 199 / 202 (forward) and 144 /
// 150 / 149 / 153 us (backward, profiles/r03_stamps_v3.log), the launch tails fell from 20-25 to
// 12 us and S10 went 820 -> 846-854 it/s (profiles/r03_assign_ab_v3.txt); the speeds below are
// that run's, corrected once more by its finish times.  [forward (both variants), backward][slot]
constexpr int kR0Slots = 4;
static const double kR0SlotSpeed[2][kR0Slots] = {{1.0, 0.970, 0.964, 0.914}, {1.0, 0.906, 0.856, 0.789}};

void plan_round0(Ctx &c, DFactor &d, const int64_t *kps_ptr) {
    for (int v = 0; v < 3; v++) d.agrid[v] = 0, d.aptr[v].release(), d.ameta[v].release();
    if (!d.pipelined || d.round_ptr.size() < 2) return;
    const int64_t b0 = d.round_ptr[0], nb = d.round_ptr[1] - b0;
    if (nb <= 0 || d.hmeta.size() < (size_t)(b0 + nb) * 8) return;
    int64_t grid[3] = {0, 0, 0};
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    pipe_round0(c, d, false, false, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, &grid[0]);
    pipe_round0(c, d, true, false, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, &grid[2]);
    if (kps_ptr && d.fcol16.n > 0) pipe_round0_resid(c, d, nullptr, nullptr, ResArgs{}, &grid[1]);
    for (int v = 0; v < 3; v++) {
        const int64_t G = grid[v];
        if (G <= 1 || G >= nb) continue;
        const double *k = kR0Cost[v];
        std::vector<double> cost(nb);
        for (int64_t i = 0; i < nb; i++) {
            const int32_t *m = &d.hmeta[(size_t)(b0 + i) * 8];
            const double ent = v == 2 ? m[7] - m[6] : m[5] - m[4];
            const double ke = (v == 1) ? (double)(kps_ptr[m[1]] - kps_ptr[m[0]]) : 0.0;
            cost[i] = k[0] + k[1] * (m[3] - m[2]) + k[2] * (m[1] - m[0]) + k[3] * ent + k[4] * ke;
        }
        std::vector<int64_t> ord(nb);
        for (int64_t i = 0; i < nb; i++) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return cost[a] > cost[b]; });
        // workgroups by dispatch slot (the j-th workgroup of every SIMD), each slot with its
        // relative speed; a block goes to the workgroup that would finish it first:
        // min over slots of (load + cost) / speed, the least loaded workgroup of each slot a heap top
        const int64_t per_slot = std::max<int64_t>(1, (int64_t)cus * 4);
        const int nslot = (int)std::min<int64_t>(kR0Slots, (G + per_slot - 1) / per_slot);
        // XCD affinity (option r0_xcd_chunk = K): runs of K consecutive blocks go to the
        // workgroups of one XCD (workgroup g on XCD g mod 8, the dispatcher's round robin -- a
        // speed assumption only), so the 128-byte lines two neighbouring blocks share in every
        // stream, and the input lines their perm gathers share, are fetched into one L2
        const int64_t K = c.opts.r0_xcd_chunk;
        const int nxcd = (K > 0 && G % 8 == 0) ? 8 : 1;
        using HE = std::pair<double, int32_t>;  // (load, workgroup)
        auto gt = [](const HE &a, const HE &b) { return a.first > b.first || (a.first == b.first && a.second > b.second); };
        std::vector<std::vector<HE>> heaps((size_t)nxcd * nslot);
        for (int64_t g = 0; g < G; g++)
            heaps[(size_t)(g % nxcd) * nslot + std::min<int64_t>(g / per_slot, nslot - 1)].push_back({0.0, (int32_t)g});
        for (auto &h : heaps) std::make_heap(h.begin(), h.end(), gt);
        std::vector<int32_t> owner(nb);
        for (int64_t i : ord) {
            const int x0 = nxcd > 1 ? (int)((i / K) % nxcd) * nslot : 0;
            int best = -1;
            double bt = 0.0;
            for (int s = x0; s < x0 + nslot; s++) {
                if (heaps[s].empty()) continue;
                const double t = (heaps[s].front().first + cost[i]) / kR0SlotSpeed[v == 2 ? 1 : 0][s - x0];
                if (best < 0 || t < bt) best = s, bt = t;
            }
            auto &h = heaps[best];
            std::pop_heap(h.begin(), h.end(), gt);
            owner[i] = h.back().second;
            h.back().first += cost[i];
            std::push_heap(h.begin(), h.end(), gt);
        }
        std::vector<int32_t> ptr((size_t)G + 1, 0), am((size_t)nb * 8);
        for (int64_t i = 0; i < nb; i++) ptr[owner[i] + 1]++;
        for (int64_t g = 0; g < G; g++) ptr[g + 1] += ptr[g];
        std::vector<int32_t> nx(ptr.begin(), ptr.end() - 1);
        for (int64_t i = 0; i < nb; i++) {  // ascending block order within a workgroup
            const int32_t q = nx[owner[i]]++;
            std::copy_n(&d.hmeta[(size_t)(b0 + i) * 8], 8, &am[(size_t)q * 8]);
        }
        d.aptr[v].upload(ptr);
        d.ameta[v].upload(am);
        d.agrid[v] = (int)G;
    }
}

template <int TPB>
static void fwd_round(Ctx &c, const DFactor &F, int64_t r, const double *xin, int64_t neg_from, double *w,
                      const int *run, const int *active, int sched_in, double *xs) {
    const int i = r == 0 ? 0 : 1;
    const int64_t b0 = F.round_ptr[r], nb = F.round_ptr[r + 1] - b0;
    if (!nb) return;
    hipLaunchKernelGGL((sptrsv_fwd_kernel<TPB>), dim3((unsigned)nb), dim3(TPB),
                       sweep_lds_bytes(F.sweep_rows[i], F.sweep_cap[i]), c.stream, b0, F.sweep_rows[i],
                       F.sweep_cap[i], (r == 0 && F.skip0) ? 1 : 0, F.blk_lvl.p, F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.perm.p,
                       xin, neg_from, w, run, active, sched_in, xs);
}

template <int TPB, bool ADD>
static void bwd_round(Ctx &c, const DFactor &F, int64_t r, double *w, double *out, const int *run,
                      const int *active, double *ys) {
    const int i = r == 0 ? 0 : 1;
    const int64_t b0 = F.round_ptr[r], nb = F.round_ptr[r + 1] - b0;
    if (!nb) return;
    hipLaunchKernelGGL((sptrsv_bwd_kernel<TPB, ADD>), dim3((unsigned)nb), dim3(TPB),
                       sweep_lds_bytes(F.sweep_rows[i], F.sweep_cap[i]), c.stream, b0, F.sweep_rows[i],
                       F.sweep_cap[i], F.blk_lvl.p, F.lvl_row.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p, F.perm.p, w,
                       out, run, active, ys);
}

static bool fwd_all(Ctx &c, const DFactor &F, const double *xin, int64_t neg_from, double *w, const int *run,
                    const int *active, int sched_in, double *xs = nullptr, int64_t rfirst = 0, FwdIn *defer = nullptr,
                    const PackArgs *pk = nullptr) {
    int64_t R = (int64_t)F.round_ptr.size() - 1;
    bool packed = pk != nullptr;  // every round launched here through a packing kernel
    if (defer && chain_ok(F, kChainFull) && rfirst <= F.chain_first) {  // the chained rounds run in the backward sweep's chain
        *defer = FwdIn{xin, neg_from, sched_in, xs, true, F.chain_first, true};
        R = F.chain_first;
        packed = false;
    } else if (defer && fuse_last_ok(F)) {  // the last round runs with the backward sweep
        *defer = FwdIn{xin, neg_from, sched_in, xs, true, R - 1};
        R -= 1;
        packed = false;  // the deferred round's rows are packed by no launch here
    }
    const PackArgs none{};
    // no deferral: the forward chain runs rounds 1 .. R-1 (distributed: the separator follows)
    const bool fchain = !(defer && defer->valid) && chain_ok(F, kChainFwd) && rfirst <= F.chain_first;
    for (int64_t r = rfirst; r < R; r++) {
        if (r == F.chain_first && fchain) {  // the chained rounds [chain_first, R)
            launch_chain(c, F, kChainFwd, FwdIn{xin, neg_from, sched_in, xs, true, r}, w, nullptr, false, run, active,
                         nullptr, pk ? *pk : none);
            break;
        }
        bool used = true;
        if (r == 0 &&
            pipe_round0(c, F, false, false, xin, neg_from, w, nullptr, run, active, sched_in, nullptr, xs, nullptr, pk,
                        &used)) {
            packed = packed && used;
            continue;
        }
        if (r > 0 &&
            upper_round(c, F, r, false, false, xin, neg_from, w, nullptr, run, active, sched_in, nullptr, xs,
                        pk ? *pk : none))
            continue;
        packed = false;
        switch (F.sweep_threads[r == 0 ? 0 : 1]) {
        case 32: fwd_round<32>(c, F, r, xin, neg_from, w, run, active, sched_in, xs); break;
        case 64: fwd_round<64>(c, F, r, xin, neg_from, w, run, active, sched_in, xs); break;
        case 128: fwd_round<128>(c, F, r, xin, neg_from, w, run, active, sched_in, xs); break;
        case 512: fwd_round<512>(c, F, r, xin, neg_from, w, run, active, sched_in, xs); break;
        case 1024: fwd_round<1024>(c, F, r, xin, neg_from, w, run, active, sched_in, xs); break;
        default: fwd_round<256>(c, F, r, xin, neg_from, w, run, active, sched_in, xs); break;
        }
    }
    CPK_HIP(hipGetLastError());
    return packed && (R > 0 || rfirst > 0);
}

bool launch_sptrsv_fwd(Ctx &c, const DFactor &F, const double *xin, int64_t neg_from, double *w, const int *run,
                       const int *active, bool sched_in, double *xs, FwdIn *defer, const PackArgs *pk) {
    // schedule-order input: no perm gather and no negation (neg_from applies to original indices)
    if (defer) defer->valid = false;
    return fwd_all(c, F, xin, sched_in ? INT64_MAX : neg_from, w, run, active, sched_in ? 1 : 0, xs, 0, defer, pk);
}

// diagnostic: the per-workgroup stamps of the last round-0 launch (0 unless built with
// CPK_PIPE_STAMPS); returns the number of pairs copied
int64_t debug_blk_cycles(uint64_t *out, int64_t n) {
#ifdef CPK_PIPE_STAMPS
    n = std::min<int64_t>(n, 12 * (int64_t)kBlkCycMax);
    CPK_HIP(hipDeviceSynchronize());
    CPK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blk_cyc), (size_t)n * sizeof(uint64_t)));
    return n;
#else
    (void)out, (void)n;
    return 0;
#endif
}

int debug_pipe_stamps(uint64_t *out, int npairs) {
#ifdef CPK_PIPE_STAMPS
    npairs = std::min(npairs, 16384);
    CPK_HIP(hipDeviceSynchronize());
    CPK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pipe_stamps), (size_t)npairs * 2 * sizeof(uint64_t)));
    return npairs;
#else
    (void)out, (void)npairs;
    return 0;
#endif
}

bool launch_sptrsv_fwd_resid(Ctx &c, const DFactor &F, const DMat &Kps, const double *xs, const double *y, double *r,
                             const int *run, FwdIn *defer, const PackArgs *pk, bool *packed) {
    if (defer) defer->valid = false;
    if (packed) *packed = false;
    const bool off = F.no_fused_resid;  // A/B switch: separate residual SpMV
    if (off || !F.pipelined || F.round0_rows < 0 || F.fcol16.n == 0 || F.round_ptr.size() < 2 ||
        Kps.halo())
        return false;
    // round 0: r of its rows formed in the sweep (nothing is launched unless a configuration
    // matches); the rows above round 0 by the round-0 kernel's workgroups after their blocks
    const ResArgs ra{Kps.ptr.p, Kps.col.p, Kps.val.p, y, xs, F.round0_rows, F.N};
    bool used = false;
    if (!pipe_round0_resid(c, F, r, run, ra, nullptr, pk, &used)) return false;
    const bool rest = fwd_all(c, F, r, INT64_MAX, r, run, nullptr, 1, nullptr, 1, defer, pk);
    if (packed) *packed = pk != nullptr && used && rest;
    return true;
}

bool launch_sptrsv_bwd(Ctx &c, const DFactor &F, double *w, double *out, bool add, const int *run,
                       const int *active, double *ys, const FwdIn *last, const PackArgs *pk, bool wdead) {
    if (!out && add && !ys) throw Error(CPK_ERR_ARGS, "internal: accumulating backward sweep without a base");
    int64_t R = (int64_t)F.round_ptr.size() - 1;
    bool packed = pk != nullptr && !(last && last->valid);
    const PackArgs none{};
    if (last && last->valid && last->chain) {  // the deferred chained rounds: one launch
        launch_chain(c, F, kChainFull, *last, w, out, add, run, active, ys, none);
        R = F.chain_first;
    } else if (!(last && last->valid) && chain_ok(F, kChainBwd)) {  // backward rounds R-1 .. chain_first
        launch_chain(c, F, kChainBwd, FwdIn{}, w, out, add, run, active, ys, pk ? *pk : none);
        R = F.chain_first;
    } else if (last && last->valid) {  // the deferred last round, forward and backward (sptrsv_last_kernel)
        launch_last(c, F, *last, w, out, add, run, active, ys);
        R = last->from;
    }
    for (int64_t r = R - 1; r >= 0; r--) {
        if (r == 0 && pipe_round0(c, F, true, add, nullptr, 0, w, out, run, active, wdead ? 1 : 0, ys, nullptr, nullptr, pk))
            continue;
        if (r > 0 && upper_round(c, F, r, true, add, nullptr, 0, w, out, run, active, 0, ys, nullptr, pk ? *pk : none))
            continue;
        packed = false;
        switch (F.sweep_threads[r == 0 ? 0 : 1] * 2 + (add ? 1 : 0)) {
        case 64: bwd_round<32, false>(c, F, r, w, out, run, active, ys); break;
        case 65: bwd_round<32, true>(c, F, r, w, out, run, active, ys); break;
        case 128: bwd_round<64, false>(c, F, r, w, out, run, active, ys); break;
        case 129: bwd_round<64, true>(c, F, r, w, out, run, active, ys); break;
        case 256: bwd_round<128, false>(c, F, r, w, out, run, active, ys); break;
        case 257: bwd_round<128, true>(c, F, r, w, out, run, active, ys); break;
        case 1024: bwd_round<512, false>(c, F, r, w, out, run, active, ys); break;
        case 1025: bwd_round<512, true>(c, F, r, w, out, run, active, ys); break;
        case 2048: bwd_round<1024, false>(c, F, r, w, out, run, active, ys); break;
        case 2049: bwd_round<1024, true>(c, F, r, w, out, run, active, ys); break;
        case 513: bwd_round<256, true>(c, F, r, w, out, run, active, ys); break;
        default: bwd_round<256, false>(c, F, r, w, out, run, active, ys); break;
        }
    }
    CPK_HIP(hipGetLastError());
    return packed && R > 0;
}

// ---- small helpers ---------------------------------------------------------------------------
__global__ void pack_slots_kernel(const int32_t *__restrict__ slot, int64_t n, const double *__restrict__ w,
                                  double *__restrict__ buf, const int *run) {
    if (run && *run == 0) return;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const int32_t s = slot[q];
        if (s >= 0) buf[s] = w[q];
    }
}

void launch_pack_slots(Ctx &c, const int32_t *slot, int64_t n, const double *w, double *buf, const int *run) {
    if (n <= 0) return;
    const int grid = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(pack_slots_kernel, dim3(grid), dim3(kBlock), 0, c.stream, slot, n, w, buf, run);
    CPK_HIP(hipGetLastError());
}

__global__ void sub_state_kernel(const double *__restrict__ x, int64_t neg_from, const double *__restrict__ g,
                                 int64_t N, double *__restrict__ t, const int *run) {
    if (run && *run == 0) return;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        const double xi = i >= neg_from ? -x[i] : x[i];
        t[i] = xi - g[i];
    }
}

void launch_sub_state(Ctx &c, const double *x, int64_t neg_from, const double *g, int64_t N, double *t,
                      const int *run) {
    if (N <= 0) return;
    const int grid = (int)std::min<int64_t>((N + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(sub_state_kernel, dim3(grid), dim3(kBlock), 0, c.stream, x, neg_from, g, N, t, run);
    CPK_HIP(hipGetLastError());
}

__global__ void set_concat_kernel(double *dst, const double *a, int64_t na, int64_t nb) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < na + nb; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = i < na ? a[i] : 0.0;
}

void launch_set_concat(Ctx &c, double *dst, const double *a, int64_t na, int64_t nb) {
    int64_t tot = na + nb;
    if (!tot) return;
    int grid = (int)std::min<int64_t>((tot + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(set_concat_kernel, dim3(grid), dim3(kBlock), 0, c.stream, dst, a, na, nb);
    CPK_HIP(hipGetLastError());
}

}  // namespace cpk
