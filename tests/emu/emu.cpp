// Host emulation of decode v28's per-lane code with the REAL functions of loona_amd/csrc (extracted
// by tests/emu/extract.py; tests/emu/shim.h stands in for the HIP builtins), against the oracle:
//   1. the wave kernel's lane protocol (hpk_wave.h): body steps (lit12_body) for a lane's first
//      literal, then its second, then both tails with checked steps that stop once a step proves the
//      end (lit12_step<.., kMore>), LUT3 and LUT2 layouts, exact-bound regions back to back, lanes in
//      reverse order (a stray byte past a region would hit an already decoded neighbour);
//   2. the fill kernel's protocol (hpk_decode12.h: LUT2, no second-byte offset stores);
//   3. hpk_decode_tiny (hpk_tiny.h) lane by lane: exact-bound and below-bound regions
//      (HPK_OUTPUT_OVERFLOW), unaligned bases, bad offsets.
// Test infrastructure only (tests/test_walk_emulation.py). Exit status 0 = no mismatch.
#include "walk.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
extern "C" int oracle_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
extern "C" int oracle_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
emu_dim3 threadIdx, blockIdx;
using namespace hpkdec;

static hpk_tables T;

static std::vector<std::vector<uint8_t>> make_lits(std::mt19937_64& rng, int nlit, int maxlen) {
    std::vector<std::vector<uint8_t>> lits;
    const char* text = "abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:ABC ";
    const char* five = "012aceiost";
    for (int i = 0; i < nlit; ++i) {
        int kind = rng() % 8, n = rng() % (maxlen + 1);
        std::vector<uint8_t> s(n);
        for (auto& c : s) c = kind == 0 ? five[rng() % 10] : kind == 1 ? text[rng() % strlen(text)] : (uint8_t)rng();
        std::vector<uint8_t> enc(4 * n + 8);
        size_t el = 0;
        if (kind <= 2 || kind >= 6) {
            oracle_encode(s.data(), n, enc.data(), enc.size(), &el);
            enc.resize(el);
        } else {
            enc = s;  // random bytes: padding errors, EOS, long codes
        }
        if (kind == 4 && enc.size() > 2) enc[enc.size() - 1] &= 0xF0;
        if (kind == 5 && enc.size() > 4) {
            size_t p = rng() % (enc.size() - 3);
            enc[p] = enc[p + 1] = enc[p + 2] = enc[p + 3] = 0xFF;
        }
        if (kind == 7) enc.push_back(0xFF);  // too much padding
        lits.push_back(enc);
    }
    return lits;
}

// kWave: the wave kernel's form (second byte stored through the +1 offset), else the fill kernel's
template <int kTab, bool kWave>
static int run_lanes(std::mt19937_64& rng, int nlit, int maxlen) {
    auto lits = make_lits(rng, nlit, maxlen);
    int bad = 0;
    for (size_t f = 0; f < lits.size(); f += 128) {
        const size_t k = std::min<size_t>(128, lits.size() - f);
        const uint32_t mis = rng() % 16;
        std::vector<uint8_t> win(mis);
        std::vector<uint32_t> p0(k), nb(k), o0(k), cap(k);
        uint32_t op = rng() % 4;
        for (size_t t = 0; t < k; ++t) {
            p0[t] = win.size();
            nb[t] = lits[f + t].size();
            win.insert(win.end(), lits[f + t].begin(), lits[f + t].end());
            o0[t] = op;
            cap[t] = nb[t] * 8 / 5;
            op += cap[t];
        }
        win.resize(win.size() + 64, 0x5A);
        std::vector<uint32_t> w32(win.size() / 4 + 4, 0);
        for (size_t j = 0; j + 4 <= win.size(); j += 4)
            w32[j / 4] = ((uint32_t)win[j] << 24) | ((uint32_t)win[j + 1] << 16) | ((uint32_t)win[j + 2] << 8) | win[j + 3];
        std::vector<uint8_t> img(op + 256 + 64, 0xEE);
        const uint32_t dmy = op + 64 + 4;  // the lane's dummy dword, past the regions
        std::vector<uint32_t> olen(k), ost(k);
        const uint32_t* lut = kTab == 3 ? T.lut3 : T.lut2;
        for (int lane = 63; lane >= 0; --lane) {
            const uint32_t t1 = lane, t2 = 127 - lane;
            auto load = [&](Lit12& Z, uint32_t tt) {
                const uint32_t u = std::min<uint32_t>(tt, k - 1);
                Z.act = tt < k;
                Z.idx = tt;
                Z.X = p0[u] * 8u + 31u;
                Z.Eb = Z.X + (Z.act ? nb[u] * 8u : 0u);
                Z.o = o0[u];
                Z.o0 = o0[u];
                Z.st = HPK_OK;
                Z.prog = false;
                lit12_load(Z, w32.data());
            };
            Lit12 L, N;
            load(L, t1);
            load(N, t2);
            bool body = L.Eb - L.X >= kBodyMin;
            while (body) lit12_body<kPred, kTab>(L, w32.data(), lut, T.lo, img.data(), body);
            Lit12 A = L;
            L = N;
            body = L.Eb - L.X >= kBodyMin;
            while (body) lit12_body<kPred, kTab>(L, w32.data(), lut, T.lo, img.data(), body);
            N = L;
            L = A;  // restored as the kernels do: Eb from the queue entry, window reloaded at X
            const uint32_t u1 = std::min<uint32_t>(t1, k - 1);
            L.Eb = L.st != HPK_OK ? L.X : p0[u1] * 8u + 31u + (L.act ? nb[u1] * 8u : 0u);
            lit12_load(L, w32.data());
            L.more = L.Eb - L.X >= 5u;
            N.more = N.Eb - N.X >= 5u;
            for (int guard = 0; (L.more || N.more) && guard < 1000000; ++guard) {
                if (L.more) lit12_step<kPred, kWave, kTab, true>(L, w32.data(), lut, T.lo, img.data(), kWave ? dmy : dmy);
                if (N.more) lit12_step<kPred, kWave, kTab, true>(N, w32.data(), lut, T.lo, img.data(), dmy);
            }
            if (L.act) olen[t1] = L.o - L.o0, ost[t1] = lit12_status(L);
            if (N.act) olen[t2] = N.o - N.o0, ost[t2] = lit12_status(N);
        }
        for (size_t t = 0; t < k; ++t) {
            std::vector<uint8_t> ref(cap[t] + 8);
            size_t rl = 0;
            const int rs = oracle_decode(lits[f + t].data(), nb[t], ref.data(), ref.size(), &rl);
            const bool ok = rs == (int)ost[t] && rl == olen[t] && memcmp(ref.data(), img.data() + o0[t], rl) == 0;
            if (!ok && bad < 5)
                printf("lanes tab %d wave %d: literal %zu (%u B): status %u vs %d, length %u vs %zu\n", kTab, (int)kWave,
                       f + t, nb[t], ost[t], rs, olen[t], rl);
            bad += !ok;
        }
        for (uint32_t j = op; j < op + 64; ++j)
            if (img[j] != 0xEE) {
                if (bad < 5) printf("lanes tab %d: byte %u past the last region written\n", kTab, j);
                ++bad;
                break;
            }
    }
    return bad;
}

static int run_tiny(std::mt19937_64& rng, int nlit, int maxlen, bool below, bool badoff) {
    auto lits = make_lits(rng, nlit, maxlen);
    const uint32_t in_mis = rng() % 16, out_mis = rng() % 16;
    std::vector<uint8_t> inb(16 + in_mis), outb;
    std::vector<uint32_t> in_off(nlit + 1), out_off(nlit + 1);
    uint32_t op = 0;
    std::vector<uint32_t> cap(nlit);
    for (int i = 0; i < nlit; ++i) {
        in_off[i] = inb.size() - 16 - in_mis;
        inb.insert(inb.end(), lits[i].begin(), lits[i].end());
        const uint32_t bnd = lits[i].size() * 8 / 5;
        cap[i] = below && bnd ? (uint32_t)(rng() % (bnd + 1)) : bnd;
        out_off[i] = op;
        op += cap[i];
    }
    in_off[nlit] = inb.size() - 16 - in_mis;
    out_off[nlit] = op;
    inb.resize(inb.size() + 64, 0x5A);
    const int jbad = badoff ? (int)(rng() % nlit) : -1;
    if (badoff) in_off[jbad] = in_off[jbad + 1] + 3;  // decreasing
    outb.assign(16 + out_mis + op + 64, 0xEE);
    std::vector<uint32_t> ol(nlit, 7);
    std::vector<uint8_t> st(nlit, 9);
    uint32_t err = 0;
    DecodeArgs a = {};
    a.in_base = inb.data() + 16;  // (the vectors' data are 16-byte aligned: new[] of >= 16 B)
    a.in_mis = in_mis;
    a.in_off = in_off.data();
    a.n = nlit;
    a.out_base = outb.data() + 16;
    a.out_mis = out_mis;
    a.out_off = out_off.data();
    a.out_len = ol.data();
    a.status = st.data();
    a.lo = T.lo;
    a.lut2 = T.lut2;
    a.in_cap = in_off[nlit];
    a.out_cap = op;
    a.err = &err;
    for (uint32_t b = 0; b < (uint32_t)(nlit + 63) / 64; ++b)
        for (uint32_t l = 0; l < 64; ++l) {
            blockIdx.x = b;
            threadIdx.x = l;
            hpk_decode_tiny(a);
        }
    int bad = 0;
    for (int i = 0; i < nlit; ++i) {
        if (badoff && i == jbad - 1) continue;  // (valid offsets, but its bytes changed with in_off[jbad])
        if (badoff && i == jbad) {
            if (!(st[i] == HPK_BAD_OFFSETS && ol[i] == 0 && err == 1)) {
                if (bad < 5) printf("tiny: bad offsets of literal %d not reported\n", i);
                ++bad;
            }
            continue;
        }
        std::vector<uint8_t> ref(lits[i].size() * 8 / 5 + 8);
        size_t rl = 0;
        int rs = oracle_decode(lits[i].data(), lits[i].size(), ref.data(), ref.size(), &rl);
        const uint8_t* got = outb.data() + 16 + out_mis + out_off[i];
        bool ok;
        if (rl <= cap[i])
            ok = st[i] == rs && ol[i] == rl && memcmp(got, ref.data(), rl) == 0;
        else  // the reference's output does not fit: the walk stops at the first byte past the capacity
            ok = st[i] == HPK_OUTPUT_OVERFLOW && ol[i] == cap[i] && memcmp(got, ref.data(), cap[i]) == 0;
        if (!ok && bad < 5)
            printf("tiny: literal %d (%zu B, cap %u): status %u vs %d, length %u vs %zu\n", i, lits[i].size(), cap[i],
                   st[i], rs, ol[i], rl);
        bad += !ok;
    }
    for (uint32_t j = 0; j < outb.size(); ++j)
        if ((j < 16 + out_mis || j >= 16 + out_mis + op) && outb[j] != 0xEE) {
            if (bad < 5) printf("tiny: guard byte %u (of %zu, regions [%u, %u)) written, below %d badoff %d\n", j,
                                outb.size(), 16 + out_mis, 16 + out_mis + op, (int)below, (int)badoff);
            ++bad;
        }
    return bad;
}

int main(int argc, char** argv) {
    if (hpk_build_tables(&T)) {
        printf("table build failed\n");
        return 1;
    }
    std::mt19937_64 rng(argc > 1 ? atoi(argv[1]) : 1);
    const int iters = argc > 2 ? atoi(argv[2]) : 8;
    int bad = 0;
    for (int it = 0; it < iters; ++it) {
        const int maxlen = (it % 3 == 0) ? 400 : 70;
        bad += run_lanes<3, true>(rng, 3000, maxlen);
        bad += run_lanes<2, true>(rng, 3000, maxlen);
        bad += run_lanes<2, false>(rng, 3000, maxlen);
        bad += run_tiny(rng, 3000, maxlen, false, false);
        bad += run_tiny(rng, 3000, maxlen, true, false);
        bad += run_tiny(rng, 500, maxlen, false, true);
    }
    printf("%s: %d mismatches\n", bad ? "FAIL" : "ok", bad);
    return bad != 0;
}
