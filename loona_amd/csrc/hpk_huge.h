// hpk_huge.h — huge-literal phase (decode v29): a literal of >= HPK_HUGE_MIN encoded bytes is decoded
// by up to a whole workgroup at once, in pieces, instead of by one lane of the long-literal phase.
//
// Why: one lane walks ~20 bits per ~600 cycles, so the long-literal phase took 125 ms for a 1 MiB
// literal where one CPU thread of the reference takes a few ms. Huffman codes do
// not mark their boundaries, so a piece that starts in the middle of a literal does not know where
// its first code starts; the walk is speculative and checked afterwards:
//   1. count: piece k of P (PB bytes each) walks from OV bits before its start (a code boundary
//      only by luck) to the first code that starts at or after its start (S_k), then counts the codes
//      that start in [S_k, start of piece k + 1) and stops at the first one that starts at or after
//      that (E_k). A walk resynchronises with the true one within a few dozen bits on header text
//      (scripts/sync_stats.py: 95 % within 128 bits), so S_k is the true boundary almost always.
//      Piece 0 starts at bit 0 (exact); the last piece walks to the literal's end;
//   2. fix: piece k is right iff S_k == E_{k-1} (its predecessor right). A piece that does not match
//      walks again from E_{k-1} (no lead); repeated until no piece changes (each round fixes at least
//      the first mismatch for good, and mismatches are rare and isolated);
//   3. the first piece that ends the walk — a code that does not fit (the literal's end, or
//      PaddingTooLarge), EOS — is the literal's last (t); pieces after it are ignored;
//   4. a scan of the counts of pieces 0..t gives each piece its output offset, and the pieces walk
//      again from S_k and store their codes (8-byte stores of whole groups, the two partial groups at a
//      piece's ends bytewise); piece t stores the length and status.
// Several huge literals share a round (a contiguous run of lanes each); rounds repeat until the
// workgroup's list is done. Input is read straight from global memory, 16-byte chunks one ahead of
// the walk. Semantics are the lane walk's (huffman.rs:95-161): a code that runs past the end stops the
// walk, EOS is EOSInString at once, then > 7 residual bits PaddingTooLarge, non-ones InvalidPadding.
// The per-piece functions are plain per-lane code (tests/emu replays them on the CPU).
#pragma once
// (included by hpk_decode12.h after the lane-walk helpers it uses: residual_status, lo_decode)

namespace hpkdec {

#ifndef HPK_HUGE_MIN
#define HPK_HUGE_MIN 8192u  // encoded bytes from which a literal is a huge one (config 3's longest: 3.4 KiB)
#endif
constexpr uint32_t kHugePieceMin = 64;  // bytes per piece at least
constexpr uint32_t kHugeTerm = 0x100u;  // piece flag: the walk ended in this piece (status in the low byte)
constexpr uint32_t kHugeNone = 0xFFFFFFFFu;
constexpr uint32_t kHugeLimit = 1u << 28;  // literal bit positions fit in 32 bits below this many bytes

// Walker over a literal in global memory: a 64-bit window (MSB first), the chunk holding the next
// dword to merge (c0) and the one after it (c1, loaded when c0 becomes current).
struct HugeWalk {
    uint64_t win;
    uint32_t nb;   // bits in win
    uint32_t qi;   // absolute dword index of the next dword to merge
    uint32_t pos;  // literal-relative bit position of win's first bit
    uint4 c0, c1;
};

// Dword j (0..3) of a chunk, by shifts: written as selects of its elements, the compiler made it a
// dynamically indexed vector access, kept the chunks in scratch memory and read them back from there.
__device__ __forceinline__ uint32_t huge_sel(const uint4& c, uint32_t j) {
    const uint32_t sh = (j & 1u) * 32u;
    const uint32_t lo = (uint32_t)((((uint64_t)c.y << 32) | c.x) >> sh);
    const uint32_t hi = (uint32_t)((((uint64_t)c.w << 32) | c.z) >> sh);
    return (j & 2u) ? hi : lo;
}

// ld16(ci): 16-byte chunk ci of the input (clamped to the batch's last chunk).
template <class Ld>
__device__ __forceinline__ void huge_begin(HugeWalk& W, const Ld& ld16, uint32_t lbyte, uint32_t pos) {
    const uint32_t b = lbyte + (pos >> 3);
    const uint32_t qd = b >> 2;
    const uint32_t sk = (b & 3u) * 8u + (pos & 7u);
    W.c0 = ld16(qd >> 2);
    W.c1 = ld16((qd >> 2) + 1u);
    W.win = ((uint64_t)hpk_bswap32(huge_sel(W.c0, qd & 3u)) << 32) << sk;
    W.nb = 32u - sk;
    W.qi = qd + 1u;
    W.pos = pos;
    if ((W.qi & 3u) == 0u) {
        W.c0 = W.c1;
        W.c1 = ld16((W.qi >> 2) + 1u);
    }
}

// The next code at W.pos (>= 33 bits in the window after the refill): symbol, length, EOS; and when
// the table entry holds a second code too, its symbol and the two codes' length (held; else 0).
template <int kTab, class Ld>
__device__ __forceinline__ void huge_peek(HugeWalk& W, const Ld& ld16, const uint32_t* __restrict__ lut,
                                          const uint16_t* __restrict__ lo, uint32_t& sym, uint32_t& len, bool& eos,
                                          uint32_t& sym1, uint32_t& held) {
    if (W.nb <= 32u) {
        W.win |= (uint64_t)hpk_bswap32(huge_sel(W.c0, W.qi & 3u)) << (32u - W.nb);
        W.nb += 32u;
        W.qi += 1u;
        if ((W.qi & 3u) == 0u) {
            W.c0 = W.c1;
            W.c1 = ld16((W.qi >> 2) + 1u);
        }
    }
    const uint32_t w = (uint32_t)(W.win >> 32);
    const uint32_t e = lut[w >> (32 - HPK_LUT_BITS)];
    const uint32_t l0 = kTab == 3 ? HPK_L3_LEN0(e) : HPK_L2_LEN0(e);  // 15: no code of <= 12 bits
    if (l0 <= (uint32_t)HPK_LUT_BITS) {
        sym = e & 0xFFu;
        len = l0;
        eos = false;
        const uint32_t codes = kTab == 3 ? HPK_L3_CODES(e) : HPK_L2_CODES(e);
        held = codes == 2u ? (kTab == 3 ? HPK_L3_HELD(e) : HPK_L2_HELD(e)) : 0u;
        sym1 = (e >> 16) & 0xFFu;
    } else {
        lo_decode(w, lo, sym, len, eos);
        held = 0;
        sym1 = 0;
    }
}

__device__ __forceinline__ void huge_adv(HugeWalk& W, uint32_t len) {
    W.win <<= len;
    W.nb -= len;
    W.pos += len;
}

// Count the codes from W.pos up to the first code that starts at or after nx (last: to the walk's
// end). c: codes counted; returns the flag (kHugeTerm | status if the walk ended here, else 0).
template <int kTab, class Ld>
__device__ __forceinline__ uint32_t huge_count(HugeWalk& W, const Ld& ld16, const uint32_t* __restrict__ lut,
                                               const uint16_t* __restrict__ lo, uint32_t nbits, uint32_t nx, bool last,
                                               uint32_t& c) {
    c = 0;
    for (;;) {
        if (!last && W.pos >= nx) return 0u;
        uint32_t sym, len, sym1, held;
        bool eos;
        huge_peek<kTab>(W, ld16, lut, lo, sym, len, eos, sym1, held);
        const uint32_t rem = nbits - W.pos;
        if (held != 0u && held <= rem && (last || W.pos + len < nx)) {  // two codes, both counted here
            huge_adv(W, held);
            c += 2u;
            continue;
        }
        if (len > rem) return kHugeTerm | residual_status(rem, (uint32_t)(W.win >> 32));  // huffman.rs:128-160
        if (eos) return kHugeTerm | HPK_EOS_IN_STRING;                                  // huffman.rs:112-116
        huge_adv(W, len);
        c += 1u;
    }
}

// Piece geometry of a literal of nbytes: P pieces of PB bytes (the last one shorter, never empty),
// OV bits of lead before a piece's start.
__device__ __forceinline__ void huge_geometry(uint32_t nbytes, uint32_t lanes, uint32_t& P, uint32_t& PB, uint32_t& OV) {
    P = min(lanes, (nbytes + kHugePieceMin - 1u) / kHugePieceMin);
    PB = (nbytes + P - 1u) / P;
    P = (nbytes + PB - 1u) / PB;
    OV = PB >= 512u ? 512u : 256u;
}

// Pass 1 of piece k: S (first code start >= the piece's start; kHugeNone if the lead walk ended
// before it), E, c, flag.
template <int kTab, class Ld>
__device__ __forceinline__ void huge_pass1(const Ld& ld16, const uint32_t* __restrict__ lut, const uint16_t* __restrict__ lo,
                                           uint32_t lbyte, uint32_t nbytes, uint32_t k, uint32_t P, uint32_t PB,
                                           uint32_t OV, uint32_t& S, uint32_t& E, uint32_t& c, uint32_t& fl) {
    const uint32_t nbits = nbytes * 8u, st = k * PB * 8u;
    const bool last = k + 1u == P;
    const uint32_t nx = last ? nbits : (k + 1u) * PB * 8u;
    HugeWalk W;
    huge_begin(W, ld16, lbyte, k == 0u ? 0u : (st > OV ? st - OV : 0u));
    c = 0;
    fl = 0;
    while (W.pos < st) {  // the lead: codes before the piece's start, not counted
        uint32_t sym, len, sym1, held;
        bool eos;
        huge_peek<kTab>(W, ld16, lut, lo, sym, len, eos, sym1, held);
        if (held != 0u && held <= nbits - W.pos && W.pos + len < st) {  // two codes, both before the start
            huge_adv(W, held);
            continue;
        }
        if (len > nbits - W.pos || eos) {  // (a speculative walk that ends: the fix walks this piece again)
            S = E = kHugeNone;
            return;
        }
        huge_adv(W, len);
    }
    S = W.pos;
    fl = huge_count<kTab>(W, ld16, lut, lo, nbits, nx, last, c);
    E = W.pos;
}

// The fix: piece k walked again from `from` (its predecessor's E).
template <int kTab, class Ld>
__device__ __forceinline__ void huge_refix(const Ld& ld16, const uint32_t* __restrict__ lut, const uint16_t* __restrict__ lo,
                                           uint32_t lbyte, uint32_t nbytes, uint32_t k, uint32_t P, uint32_t PB,
                                           uint32_t from, uint32_t& S, uint32_t& E, uint32_t& c, uint32_t& fl) {
    const uint32_t nbits = nbytes * 8u;
    const bool last = k + 1u == P;
    const uint32_t nx = last ? nbits : (k + 1u) * PB * 8u;
    HugeWalk W;
    huge_begin(W, ld16, lbyte, from);
    S = from;
    fl = huge_count<kTab>(W, ld16, lut, lo, nbits, nx, last, c);
    E = W.pos;
}

// Pass 2 of a piece: its c codes from S, stored at output byte ob (absolute, out_base-relative):
// 8-byte stores of the whole 8-byte groups, the partial groups at the two ends bytewise.
template <int kTab, class Ld, class St8, class St1>
__device__ __forceinline__ void huge_pass2(const Ld& ld16, const uint32_t* __restrict__ lut, const uint16_t* __restrict__ lo,
                                           uint32_t lbyte, uint32_t S, uint32_t c, uint32_t ob, const St8& st8,
                                           const St1& st1) {
    HugeWalk W;
    huge_begin(W, ld16, lbyte, S);
    uint64_t acc = 0;
    uint32_t p = ob;
    auto emit = [&](uint32_t sym) {
        acc |= (uint64_t)sym << (8u * (p & 7u));
        if ((p & 7u) == 7u) {
            const uint32_t g = p - 7u;
            if (g >= ob) {
                st8(g, acc);
            } else {
                for (uint32_t x = ob; x <= p; ++x) st1(x, (uint8_t)(acc >> (8u * (x & 7u))));
            }
            acc = 0;
        }
        p += 1u;
    };
    for (uint32_t j = 0; j < c;) {
        uint32_t sym, len, sym1, held;
        bool eos;
        huge_peek<kTab>(W, ld16, lut, lo, sym, len, eos, sym1, held);
        emit(sym);
        if (held != 0u && j + 2u <= c) {  // (the codes pass 1 counted: both exist)
            emit(sym1);
            huge_adv(W, held);
            j += 2u;
        } else {
            huge_adv(W, len);
            j += 1u;
        }
    }
    for (uint32_t x = max(ob, p & ~7u); x < p; ++x) st1(x, (uint8_t)(acc >> (8u * (x & 7u))));
}

}  // namespace hpkdec

#ifndef HPK_HUGE_HOST  // (tests/emu: the per-piece functions only)
namespace hpkdec {

// The phase: all kBlock threads of the workgroup call it (after the fills, before the long-literal
// phase), with the workgroup's list s_list[0, cnt) of huge literals (validated when listed: offsets in
// bounds, regions >= the decoded bound) and a scratch area of LDS (kHugeLds bytes, 16-byte aligned).
template <int kBlock>
constexpr int huge_lds_bytes() {
    return 3 * kBlock * 4 + (5 * kHugeMax + 4 + 16) * 4;
}

template <int kBlock, int kTab>
__device__ void huge_phase(const DecodeArgs& a, const uint32_t* s_list, uint32_t cnt, uint32_t* meta,
                           const uint32_t* __restrict__ s_lut, const uint16_t* __restrict__ s_lo) {
    if (cnt == 0) return;  // (block-uniform)
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    uint32_t* const mE = meta;               // per piece: E and flag (read by the next piece), scan
    uint32_t* const mF = meta + kBlock;
    uint32_t* const mX = meta + 2 * kBlock;
    uint32_t* const jl = meta + 3 * kBlock;  // jobs: literal, first lane, pieces, terminal piece
    uint32_t* const jb = jl + kHugeMax;
    uint32_t* const jp = jb + kHugeMax;
    uint32_t* const jt = jp + kHugeMax;
    uint32_t* const jo = jt + kHugeMax;      // output offset (out_base-relative, before out_mis)
    uint32_t* const jm = jo + kHugeMax;      // [0] jobs, [1] next list entry, [2] lanes used, [3..4] fix flags
    uint32_t* const wt = jm + 4;             // wave totals of the scan
    const uint32_t in_end = min(a.in_off[a.n], a.in_cap) + a.in_mis;
    const uint32_t last16 = in_end ? (in_end - 1u) >> 4 : 0u;
    const uint4* const g16 = reinterpret_cast<const uint4*>(a.in_base);
    auto ld16 = [&](uint32_t ci) { return g16[min(ci, last16)]; };
    uint8_t* const out = a.out_base;
    auto st8 = [&](uint32_t g, uint64_t v) { *reinterpret_cast<uint64_t*>(out + g) = v; };
    auto st1 = [&](uint32_t x, uint8_t v) { out[x] = v; };
    for (uint32_t cur = 0; cur < cnt;) {  // block-uniform
        __syncthreads();
        if (tid == 0) {  // the round's jobs: literals from the list while their pieces fit the block
            uint32_t nj = 0, used = 0, e = cur;
            for (; e < cnt && nj < kHugeMax; ++e) {
                const uint32_t i = s_list[e];
                const uint32_t nb = a.in_off[i + 1] - a.in_off[i];
                uint32_t P, PB, OV;
                huge_geometry(nb, kBlock, P, PB, OV);
                if (used + P > (uint32_t)kBlock) break;
                jl[nj] = i;
                // (the compacted mode, a.cursor set: the literal's decoded bound from the cursor, now)
                jo[nj] = a.cursor ? atomicAdd(a.cursor, (nb * 8u) / 5u) : a.lit_out[i];
                if (a.cursor) a.co_off[i] = jo[nj];
                jb[nj] = used;
                jp[nj] = P;
                jt[nj] = kHugeNone;
                used += P;
                ++nj;
            }
            jm[0] = nj;
            jm[1] = e;
            jm[2] = used;
            jm[3] = 0;
        }
        __syncthreads();
        const uint32_t nj = jm[0], used = jm[2];
        cur = jm[1];
        const bool on = tid < used;
        uint32_t j = 0;
        for (uint32_t q = 1; q < nj; ++q) j = jb[q] <= tid ? q : j;
        const uint32_t i = jl[j], base = jb[j], obase = jo[j];
        const uint32_t k = tid - base;
        const uint32_t p0 = a.in_off[i], nbytes = a.in_off[i + 1] - p0;
        const uint32_t lbyte = p0 + a.in_mis;
        uint32_t P, PB, OV;
        huge_geometry(nbytes, kBlock, P, PB, OV);
        uint32_t S = 0, E = 0, c = 0, fl = 0;
        if (on) {
            huge_pass1<kTab>(ld16, s_lut, s_lo, lbyte, nbytes, k, P, PB, OV, S, E, c, fl);
            mE[tid] = E;
            mF[tid] = fl;
        }
        // the fix rounds: "any piece re-walks" through a pair of LDS flags (round r sets flag r % 2 and
        // clears the other, which every thread has read before this round's first barrier)
        for (uint32_t r = 0;; ++r) {
            __syncthreads();
            bool need = false;
            uint32_t from = 0;
            if (on && k > 0u) {
                const uint32_t pe = mE[tid - 1], pf = mF[tid - 1];
                need = !(pf & kHugeTerm) && pe != kHugeNone && S != pe;
                from = pe;
            }
            if (tid == 0) jm[3 + ((r + 1u) & 1u)] = 0;
            if (need) jm[3 + (r & 1u)] = 1;
            __syncthreads();
            if (jm[3 + (r & 1u)] == 0u) break;
            if (need) {
                huge_refix<kTab>(ld16, s_lut, s_lo, lbyte, nbytes, k, P, PB, from, S, E, c, fl);
                mE[tid] = E;
                mF[tid] = fl;
            }
        }
        if (on && (fl & kHugeTerm)) atomicMin(&jt[j], k);
        __syncthreads();
        const uint32_t t = on ? jt[j] : 0u;
        const bool live = on && k <= t;
        // exclusive scan of the live pieces' counts over the block
        const uint32_t v = live ? c : 0u;
        uint32_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (lane >= (uint32_t)d) x += y;
        }
        if (lane == 63u) wt[wv] = x;
        __syncthreads();
        uint32_t pre = 0;
        for (uint32_t q = 0; q < wv; ++q) pre += wt[q];
        const uint32_t ex = pre + x - v;
        mX[tid] = ex;
        __syncthreads();
        if (live) {
            const uint32_t D = ex - mX[base];
            huge_pass2<kTab>(ld16, s_lut, s_lo, lbyte, S, c, obase + a.out_mis + D, st8, st1);
            if (k == t) {
                a.out_len[i] = D + c;
                a.status[i] = (uint8_t)(fl & 0xFFu);
            }
        }
    }
    __syncthreads();
}

}  // namespace hpkdec
#endif
