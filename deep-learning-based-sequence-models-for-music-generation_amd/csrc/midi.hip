// Token -> note decode of generated MIDI-token rows (processing/processing.py
// :171-214 decode, + :154-169 revert_note_time), run on the device right after
// the sampler so the B generated rows never leave HBM as token ids.
//
// The reference walks a row token by token: each token sets one field (pitch
// + channel, dyn, length, time shift, tempo); a note is emitted when pitch,
// dyn, length and tempo have all been set since the previous note (the time
// shift persists), then those four fields are cleared. Note starts are the
// running sum of the time shifts, in beats; revert_note_time then maps beats
// to seconds with a running fp64 sum that uses the PREVIOUS note's tempo.
//
// Four wavefronts per row (one workgroup), integer/byte work (no MFMA):
//  * the "fields seen since the last note" state is a 4-bit mask, so the
//    reference's sequential walk is a 16-state automaton; each lane folds its
//    chunk of tokens into a transition map for all 16 start states at once
//    (16 nibbles of one uint64, updated with bit ops), and a wave scan of map
//    composition (waves, then the 4 wave totals through LDS) gives every
//    thread its exact start state;
//  * field values at an emission are the last token of each class up to that
//    point (a max-scan of positions), time shifts and note counts are
//    exclusive wave sums;
//  * the fp64 beat->seconds recurrence is kept sequential in the reference's
//    own operation order (bit-identical doubles): per 64-note batch every lane
//    computes its increment, then a 64-step readlane chain adds them.
#include "common.h"

namespace {

constexpr int MIDI_WAVES = 4, MIDI_NT = 64 * MIDI_WAVES;  // 4 wavefronts share one row
// chunk stride csp = cs | 1 <= 63 keeps the staged row (+ the wave totals) within 64 KB of LDS
constexpr int64_t MIDI_MAX_L = MIDI_NT * 62;

struct Disc {
    int64_t P, dyn0, len0, time0, tempo0;
};

// token class: 0 pitch, 1 dyn, 2 length, 3 time, 4 tempo (processing.py:183-194)
__device__ __forceinline__ int tok_class(int64_t t, const Disc& d) {
    return t < d.dyn0 ? 0 : t < d.len0 ? 1 : t < d.time0 ? 2 : t < d.tempo0 ? 3 : 4;
}
// bit in the "seen" mask; time shifts do not take part
__device__ __forceinline__ uint64_t class_bit(int c) { return c == 3 ? 0 : c == 4 ? 8 : (1u << c); }

constexpr uint64_t NIB1 = 0x1111111111111111ull;
constexpr uint64_t IDENT = 0xFEDCBA9876543210ull;  // nibble s holds s

// apply one token to all 16 start states packed in m (nibble s = current state
// of the walk started in s): set the class bit, then clear states that became 15
__device__ __forceinline__ uint64_t step_all(uint64_t m, uint64_t bit) {
    m |= bit * NIB1;
    const uint64_t full = m & (m >> 1) & (m >> 2) & (m >> 3) & NIB1;
    return m & ~(full * 0xF);
}
__device__ __forceinline__ int nib(uint64_t m, int s) { return (int)((m >> (4 * s)) & 0xF); }
// (g after f)[s] = g[f[s]]
__device__ __forceinline__ uint64_t compose(uint64_t g, uint64_t f) {
    uint64_t r = 0;
#pragma unroll
    for (int s = 0; s < 16; ++s) r |= (uint64_t)nib(g, nib(f, s)) << (4 * s);
    return r;
}

__device__ __forceinline__ int64_t wave_excl_sum(int64_t v, int lane) {
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x - v;
}
__device__ __forceinline__ int64_t wave_excl_max(int64_t v, int lane) {
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x = max(x, y);
    }
    const int64_t p = __shfl_up(x, 1, 64);
    return lane == 0 ? (int64_t)-1 : p;
}

// rows [B, ld] int64 (first L tokens used); per row b the notes go to
// [b*cap, b*cap + count[b]) of pitch / channel / dyn / tempo (int32),
// beat_start / beat_end (int64, pre-revert note times) and t_start / t_end
// (fp64 seconds, revert_note_time). count[b] is the full note count even when
// it exceeds cap (only the first cap notes are written).
__global__ __launch_bounds__(MIDI_NT) void midi_decode_kernel(const int64_t* __restrict__ rows, int64_t ld, int64_t L,
                                                         int64_t cap, Disc d, double res_per_beat,
                                                         int32_t* __restrict__ pitch, int32_t* __restrict__ channel,
                                                         int32_t* __restrict__ dyn, int32_t* __restrict__ tempo,
                                                         int64_t* __restrict__ beat_start,
                                                         int64_t* __restrict__ beat_end, double* __restrict__ t_start,
                                                         double* __restrict__ t_end, int64_t* __restrict__ count) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t b = blockIdx.x;
    const int64_t* row = rows + b * ld;
    // positions fit int32 (L <= MIDI_MAX_L); no integer division inside the walks
    const int n_tok = (int)L, cs = (n_tok + MIDI_NT - 1) / MIDI_NT, csp = cs | 1;
    const int lo = min(tid * cs, n_tok), hi = min(lo + cs, n_tok);
    // the row is staged once into LDS (coalesced int64 reads, int32 tokens) in
    // lane-chunk order with an odd chunk stride, so the per-lane walks below
    // read conflict-free LDS instead of 64 scattered HBM lines per step
    extern __shared__ int32_t tok_lds[];
    // 16 coalesced loads in flight per lane (one dependent HBM round trip per
    // 1024 tokens instead of per 64); chunk of token i = i / cs via a float
    // reciprocal with an exact integer fix-up
    const float inv_cs = cs > 0 ? 1.0f / (float)cs : 0.0f;
    for (int i0 = 0; i0 < n_tok; i0 += MIDI_NT * 16) {
        int32_t v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int i = i0 + u * MIDI_NT + tid;
            v[u] = i < n_tok ? (int32_t)row[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int i = i0 + u * MIDI_NT + tid;
            if (i < n_tok) {
                int ch = (int)((float)i * inv_cs);
                ch -= ch * cs > i;
                ch += (ch + 1) * cs <= i;
                tok_lds[ch * csp + (i - ch * cs)] = v[u];
            }
        }
    }
    __syncthreads();
    const int32_t* my = tok_lds + tid * csp;  // my[j] = token lo + j

    // pass 1: transition map of this chunk + last position of every class
    uint64_t m = IDENT;
    int l0 = -1, l1 = -1, l2 = -1, l3 = -1, l4 = -1;
#pragma unroll 4
    for (int j = 0; j < hi - lo; ++j) {
        const int c = tok_class(my[j], d);
        l0 = c == 0 ? j : l0; l1 = c == 1 ? j : l1; l2 = c == 2 ? j : l2;
        l3 = c == 3 ? j : l3; l4 = c == 4 ? j : l4;
        m = step_all(m, class_bit(c));
    }
    // inclusive scan of map composition (later chunk applied after earlier)
    uint64_t inc = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t prev = __shfl_up(inc, o, 64);
        if (lane >= o) inc = compose(inc, prev);
    }
    const uint64_t before = __shfl_up(inc, 1, 64);
    // workgroup level: wave totals through LDS, each wave folds the earlier ones
    __shared__ uint64_t wg_map[MIDI_WAVES];
    __shared__ int64_t wg_last[5][MIDI_WAVES], wg_n[MIDI_WAVES], wg_td[MIDI_WAVES];
    const int64_t gl[5] = {l0 >= 0 ? (int64_t)(lo + l0) : -1, l1 >= 0 ? (int64_t)(lo + l1) : -1,
                           l2 >= 0 ? (int64_t)(lo + l2) : -1, l3 >= 0 ? (int64_t)(lo + l3) : -1,
                           l4 >= 0 ? (int64_t)(lo + l4) : -1};
    int64_t ex[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        ex[c] = wave_excl_max(gl[c], lane);
        if (lane == 63) wg_last[c][w] = max(ex[c], gl[c]);
    }
    if (lane == 63) wg_map[w] = inc;
    __syncthreads();
    uint64_t pre = IDENT;
    for (int v = 0; v < w; ++v) pre = compose(wg_map[v], pre);
    const int s0 = nib(pre, 0);
    const int state = lane == 0 ? s0 : nib(before, s0);
    // value of the last token of each class before this chunk (a max-scan of
    // global positions; -1 = none yet). Positions map back to LDS once here.
    auto carry = [&](int c) -> int64_t {
        int64_t gp = ex[c];
        for (int v = 0; v < w; ++v) gp = max(gp, wg_last[c][v]);
        if (gp < 0) return -1;
        const int ch = (int)gp / cs;
        return tok_lds[ch * csp + ((int)gp - ch * cs)];
    };
    const int64_t c0 = carry(0), c1 = carry(1), c2 = carry(2), c3 = carry(3), c4 = carry(4);

    // pass 2: notes and time-shift sum of this chunk from the exact start state
    int64_t n_loc = 0, td_loc = 0;
    {
        int st = state;
        int64_t tv = c3;
    #pragma unroll 4
    for (int j = 0; j < hi - lo; ++j) {
            const int64_t t = my[j];
            const int c = tok_class(t, d);
            tv = c == 3 ? t : tv;
            st |= (int)class_bit(c);
            if (st == 15) {
                ++n_loc;
                td_loc += tv >= 0 ? tv - d.time0 : 0;
                st = 0;
            }
        }
    }
    int64_t n_off = wave_excl_sum(n_loc, lane);
    int64_t beat_off = wave_excl_sum(td_loc, lane);
    if (lane == 63) {
        wg_n[w] = n_off + n_loc;
        wg_td[w] = beat_off + td_loc;
    }
    __syncthreads();
    int64_t n_tot = 0;
    for (int v = 0; v < MIDI_WAVES; ++v) {
        if (v < w) {
            n_off += wg_n[v];
            beat_off += wg_td[v];
        }
        n_tot += wg_n[v];
    }
    if (tid == 0) count[b] = n_tot;

    // pass 3: write the notes (integer fields and beat times)
    const int64_t base = b * cap;
    {
        int st = state;
        int64_t v0 = c0, v1 = c1, v2 = c2, v3 = c3, v4 = c4;
        int64_t k = n_off, beat = beat_off;
    #pragma unroll 4
    for (int j = 0; j < hi - lo; ++j) {
            const int64_t t = my[j];
            const int c = tok_class(t, d);
            v0 = c == 0 ? t : v0; v1 = c == 1 ? t : v1; v2 = c == 2 ? t : v2;
            v3 = c == 3 ? t : v3; v4 = c == 4 ? t : v4;
            st |= (int)class_bit(c);
            if (st == 15) {
                beat += v3 >= 0 ? v3 - d.time0 : 0;
                if (k < cap) {
                    pitch[base + k] = (int32_t)v0 % (int32_t)d.P;
                    channel[base + k] = (int32_t)v0 / (int32_t)d.P;
                    dyn[base + k] = (int32_t)(v1 - d.dyn0);
                    tempo[base + k] = (int32_t)(v4 - d.tempo0);
                    beat_start[base + k] = beat;
                    beat_end[base + k] = beat + (v2 - d.len0);
                }
                ++k;
                st = 0;
            }
        }
    }
    __syncthreads();  // workgroup-scope fence: wave 0 reads every wave's notes
    if (w != 0) return;

    // pass 4: revert_note_time (processing.py:154-169), reference operation order:
    //   res = 60 / prev_tempo / res_per_beat
    //   ts  = prev_time + (beat - prev_beat) * res ; te = ts + (beat_end - beat) * res
    const int64_t n = min(n_tot, cap);
    // raw note fields of one 64-note batch; the next batch's loads are issued
    // before the current batch's add chain so their latency hides behind it
    int32_t tp_c = 1, tp_n = 1;
    int64_t pb_c = 0, bs_c = 0, be_c = 0, pb_n = 0, bs_n = 0, be_n = 0;
    auto load = [&](int64_t k, int32_t& tp, int64_t& pb, int64_t& bs, int64_t& be) {
        if (k < n) {
            tp = tempo[base + (k == 0 ? 0 : k - 1)];
            pb = k == 0 ? 0 : beat_start[base + k - 1];
            bs = beat_start[base + k];
            be = beat_end[base + k];
        }
    };
    load(lane, tp_c, pb_c, bs_c, be_c);
    double prev_time = 0.0;
    for (int64_t k0 = 0; k0 < n; k0 += 64) {
        const int64_t k = k0 + lane;
        double inc_k = 0.0, dur_k = 0.0;
        if (k < n) {
            const double res = 60.0 / (double)tp_c / res_per_beat;
            const double bs = (double)bs_c;
            inc_k = (bs - (double)pb_c) * res;
            dur_k = ((double)be_c - bs) * res;
        }
        load(k + 64, tp_n, pb_n, bs_n, be_n);
        // the add chain reads each lane's increment with v_readlane (scalar
        // broadcast, a few cycles) instead of an LDS-crossbar shuffle per step
        const uint64_t inc_bits = __builtin_bit_cast(uint64_t, inc_k);
        const int inc_lo = (int)(uint32_t)inc_bits, inc_hi = (int)(uint32_t)(inc_bits >> 32);
        double ts = 0.0, run = prev_time;
#pragma unroll
        for (int j = 0; j < 64; ++j) {
            const uint64_t bj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(inc_lo, j) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(inc_hi, j) << 32);
            run = run + __builtin_bit_cast(double, bj);
            if (j == lane) ts = run;
        }
        if (k < n) {
            t_start[base + k] = ts;
            t_end[base + k] = ts + dur_k;
        }
        prev_time = __shfl(ts, (int)min((int64_t)63, n - 1 - k0), 64);
        tp_c = tp_n; pb_c = pb_n; bs_c = bs_n; be_c = be_n;
    }
}


// Note -> token encode of a batch of songs (processing/processing.py:129-152
// encode, + :111-126 adjust_note_time): the offline preprocessing step that
// turns extracted notes into the .npy token rows the data feed reads.
// One wavefront per song, 64 notes per step:
//  * adjust_note_time is a running fp64 sum of (start - prev_start) /
//    resolution, resolution from the PREVIOUS note's tempo: every lane forms
//    its note's increment, then a 64-step readlane chain adds them in the
//    reference's order (bit-identical doubles, FMA contraction off); int()
//    truncation gives the note's start / end beat (a note whose end truncates
//    to its start lasts one beat);
//  * the token count of a note is 4, plus 1 when its time-shift token differs
//    from the previous note's (the first note always emits one); an
//    exclusive wave sum places every note's tokens.
// Songs are independent: grid = n_songs.
__global__ __launch_bounds__(64) void midi_encode_kernel(const int32_t* __restrict__ pitch,
                                                         const int32_t* __restrict__ channel,
                                                         const int32_t* __restrict__ dyn,
                                                         const int32_t* __restrict__ tempo,
                                                         const double* __restrict__ t_start,
                                                         const double* __restrict__ t_end,
                                                         const int64_t* __restrict__ song_off, int64_t P, int64_t C,
                                                         int64_t D, int64_t Ln, int64_t Tm, int64_t Tp, Disc d,
                                                         double res_per_beat, int64_t* __restrict__ tokens,
                                                         int64_t* __restrict__ beat_start,
                                                         int64_t* __restrict__ beat_end, int64_t* __restrict__ count) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x;
    const int64_t s = blockIdx.x, o = song_off[s], n = song_off[s + 1] - o;
    int64_t* out = tokens + 5 * o;
    double run = 0.0;         // current_beats after the previous step's last note
    int64_t bs_last = 0;      // time_prev (integer beat start of the previous note)
    int64_t td_last = 0;      // time_delta_prev (a token id; 0 before the first note)
    int64_t pos = 0;          // tokens written so far
    for (int64_t k0 = 0; k0 < n; k0 += 64) {
        const int64_t k = k0 + lane;
        double inc = 0.0, dur = 0.0;
        int32_t pi = 0, ch = 0, dy = 0, tp = 0;
        if (k < n) {
            const int64_t i = o + k;
            const double prev_t = k == 0 ? 0.0 : t_start[i - 1];
            const int32_t prev_tp = k == 0 ? tempo[o] : tempo[i - 1];
            const double resolution = 60.0 / (double)prev_tp / res_per_beat;
            const double ts = t_start[i];
            inc = (ts - prev_t) / resolution;
            dur = (t_end[i] - ts) / resolution;
            pi = pitch[i];
            ch = channel[i];
            dy = dyn[i];
            tp = tempo[i];
        }
        const uint64_t ib = __builtin_bit_cast(uint64_t, inc);
        const int ilo = (int)(uint32_t)ib, ihi = (int)(uint32_t)(ib >> 32);
        double cur = 0.0, r = run;
#pragma unroll
        for (int j = 0; j < 64; ++j) {
            const uint64_t bj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(ilo, j) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(ihi, j) << 32);
            r = r + __builtin_bit_cast(double, bj);
            if (j == lane) cur = r;
        }
        const int64_t last = min((int64_t)63, n - 1 - k0);
        run = __shfl(cur, (int)last, 64);
        const double fut = cur + dur;
        const int64_t bs = (int64_t)cur;   // int(): truncation toward zero
        const int64_t fe = (int64_t)fut;
        const int64_t be = fe == bs ? bs + 1 : fe;
        // previous note's beat start / time token (lane - 1, or the carry)
        int64_t bs_prev = __shfl_up(bs, 1, 64);
        if (lane == 0) bs_prev = bs_last;
        const int64_t td = d.time0 + min(bs - bs_prev, Tm - 1);
        int64_t td_prev = __shfl_up(td, 1, 64);
        if (lane == 0) td_prev = td_last;
        const int64_t cnt = k < n ? (td != td_prev ? 5 : 4) : 0;
        const int64_t at = pos + wave_excl_sum(cnt, lane);
        if (k < n) {
            beat_start[o + k] = bs;
            beat_end[o + k] = be;
            int64_t* q = out + at;
            q[0] = min((int64_t)pi + (int64_t)ch * P, P * C - 1);  // start_idx pitch = 0
            q[1] = d.dyn0 + min((int64_t)dy, D - 1);
            q[2] = d.len0 + min(be - bs, Ln - 1);
            int e = 3;
            if (td != td_prev) q[e++] = td;
            q[e] = d.tempo0 + min((int64_t)tp, Tp - 1);
        }
        bs_last = __shfl(bs, (int)last, 64);
        td_last = __shfl(td, (int)last, 64);
        pos = __shfl(at + cnt, (int)last, 64);
    }
    if (lane == 0) count[s] = pos;
}
}  // namespace

extern "C" int msq_midi_decode(const int64_t* rows, int64_t B, int64_t L, int64_t ld, const int64_t* disc,
                               int64_t res_per_beat, int64_t cap, int32_t* pitch, int32_t* channel, int32_t* dyn,
                               int32_t* tempo, int64_t* beat_start, int64_t* beat_end, double* t_start,
                               double* t_end, int64_t* count, void* stream) {
    MSQ_CHECK_ARG(rows && B > 0 && L >= 0 && ld >= L && cap >= 0 && disc && res_per_beat > 0,
                  "msq_midi_decode: bad args");
    MSQ_CHECK_ARG(pitch && channel && dyn && tempo && beat_start && beat_end && t_start && t_end && count,
                  "msq_midi_decode: null output");
    MSQ_CHECK_ARG(L <= MIDI_MAX_L, "msq_midi_decode: row longer than %lld tokens", (long long)MIDI_MAX_L);
    // disc = {pitch, channel, dyn, length, time, tempo} (config.yaml discretization)
    Disc d{};
    d.P = disc[0];
    d.dyn0 = disc[0] * disc[1];
    d.len0 = d.dyn0 + disc[2];
    d.time0 = d.len0 + disc[3];
    d.tempo0 = d.time0 + disc[4];
    MSQ_CHECK_ARG(disc[0] > 0 && disc[1] > 0 && disc[2] > 0 && disc[3] > 0 && disc[4] > 0 && disc[5] > 0,
                  "msq_midi_decode: bad discretization");
    const size_t lds = (size_t)MIDI_NT * (((L + MIDI_NT - 1) / MIDI_NT) | 1) * sizeof(int32_t);
    hipLaunchKernelGGL(midi_decode_kernel, dim3((unsigned)B), dim3(MIDI_NT), lds, (hipStream_t)stream, rows, ld, L, cap, d,
                       (double)res_per_beat, pitch, channel, dyn, tempo, beat_start, beat_end, t_start, t_end, count);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_midi_encode(const int32_t* pitch, const int32_t* channel, const int32_t* dyn, const int32_t* tempo,
                               const double* t_start, const double* t_end, const int64_t* song_off,
                               int64_t n_songs, const int64_t* disc, int64_t res_per_beat, int64_t* tokens,
                               int64_t* beat_start, int64_t* beat_end, int64_t* count, void* stream) {
    MSQ_CHECK_ARG(n_songs >= 0 && song_off && disc && res_per_beat > 0, "msq_midi_encode: bad args");
    MSQ_CHECK_ARG(pitch && channel && dyn && tempo && t_start && t_end, "msq_midi_encode: null note column");
    MSQ_CHECK_ARG(tokens && beat_start && beat_end && count, "msq_midi_encode: null output");
    MSQ_CHECK_ARG(disc[0] > 0 && disc[1] > 0 && disc[2] > 0 && disc[3] > 0 && disc[4] > 0 && disc[5] > 0,
                  "msq_midi_encode: bad discretization");
    if (n_songs == 0) return MSQ_OK;
    Disc d{};
    d.P = disc[0];
    d.dyn0 = disc[0] * disc[1];
    d.len0 = d.dyn0 + disc[2];
    d.time0 = d.len0 + disc[3];
    d.tempo0 = d.time0 + disc[4];
    hipLaunchKernelGGL(midi_encode_kernel, dim3((unsigned)n_songs), dim3(64), 0, (hipStream_t)stream, pitch, channel, dyn,
                       tempo, t_start, t_end, song_off, disc[0], disc[1], disc[2], disc[3], disc[4], disc[5], d,
                       (double)res_per_beat, tokens, beat_start, beat_end, count);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
