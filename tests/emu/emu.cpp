// Host emulation of decode v28's per-lane code with the REAL functions of loona_amd/csrc (extracted
// by tests/emu/extract.py; tests/emu/shim.h stands in for the HIP builtins), against the oracle:
//   1. the wave kernel's lane protocol (hpk_wave.h): body steps (lit12_body) for a lane's first
//      literal, then its second, then both tails with checked steps that stop once a step proves the
//      end (lit12_step<.., kMore>), LUT3 and LUT2 layouts, exact-bound regions back to back, lanes in
//      reverse order (a stray byte past a region would hit an already decoded neighbour);
//   2. the fill kernel's protocol (hpk_decode12.h: LUT2, no second-byte offset stores);
//   3. the huge-literal phase (hpk_huge.h): its per-piece functions under the workgroup's protocol.
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

// The huge-literal phase (hpk_huge.h) piece by piece, with the workgroup's protocol replayed on the
// host (pass 1 for every piece, fix rounds on a snapshot of the pieces' ends, the first terminal piece,
// the scan, pass 2): literals of 8 KiB to 1 MiB, valid, EOS near the end or at a piece boundary, bad
// and too-long padding, random bytes, in exact-bound regions between guard bytes.
static int run_huge(std::mt19937_64& rng, int nlit, uint32_t lanes, long* fixes) {
    const char* text = "abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:ABC ";
    int bad = 0;
    for (int it = 0; it < nlit; ++it) {
        static const uint32_t sizes[] = {8192, 9001, 16384, 65535, 65536, 65537, 100003, 262144};
        uint32_t want = it == 0 ? (1u << 20) : sizes[rng() % 8];
        const int kind = rng() % 7;
        std::vector<uint8_t> enc;
        if (kind == 6) {
            enc.resize(want);
            for (auto& c : enc) c = (uint8_t)rng();
        } else {
            std::vector<uint8_t> d(want * 8 / 5 + 16);
            const bool five = kind == 1;
            for (auto& c : d) c = five ? "012aceiost"[rng() % 10] : text[rng() % strlen(text)];
            if (kind == 5)  // long codes sprinkled in (random bytes every ~300 characters)
                for (size_t q = 0; q < d.size(); q += 200 + rng() % 200) d[q] = (uint8_t)rng();
            enc.resize(4 * d.size() + 8);
            size_t el = 0;
            oracle_encode(d.data(), d.size(), enc.data(), enc.size(), &el);
            enc.resize(std::min<size_t>(el, want));  // (cut: the tail is bad padding or a cut code)
            if (kind == 2 && enc.size() > 8) {  // EOS near the end, or at a piece boundary
                size_t p = rng() % 2 ? enc.size() - 6 : (enc.size() / 2) & ~(size_t)127;
                enc[p] = enc[p + 1] = enc[p + 2] = enc[p + 3] = 0xFF;
            }
            if (kind == 3) enc.push_back(0xFF);  // padding too long
            if (kind == 4) enc.back() &= 0xF0;
        }
        const uint32_t nb = enc.size();
        const uint32_t in_mis = rng() % 16, out_mis = rng() % 16;
        std::vector<uint8_t> inb(16 + in_mis + nb + 64, 0x5A);
        memcpy(inb.data() + 16 + in_mis, enc.data(), nb);
        const uint8_t* in_base = inb.data() + 16;  // (16-byte aligned)
        const uint32_t last16 = (in_mis + nb - 1) >> 4;
        auto ld16 = [&](uint32_t ci) {
            uint4 v;
            memcpy(&v, in_base + 16 * std::min(ci, last16), 16);
            return v;
        };
        const uint32_t cap = nb * 8 / 5;
        std::vector<uint8_t> outb(16 + out_mis + cap + 64, 0xEE);
        uint8_t* out_base = outb.data() + 16;
        auto st8 = [&](uint32_t g, uint64_t v) {
            if (g % 8) printf("huge: unaligned 8-byte store\n");
            memcpy(out_base + g, &v, 8);
        };
        auto st1 = [&](uint32_t x, uint8_t v) { out_base[x] = v; };
        uint32_t P, PB, OV;
        huge_geometry(nb, lanes, P, PB, OV);
        std::vector<uint32_t> S(P), E(P), c(P), fl(P);
        for (uint32_t k = 0; k < P; ++k) huge_pass1<2>(ld16, T.lut2, T.lo, in_mis, nb, k, P, PB, OV, S[k], E[k], c[k], fl[k]);
        for (int guard = 0;; ++guard) {
            std::vector<uint32_t> from(P, kHugeNone);
            bool any = false;
            for (uint32_t k = 1; k < P; ++k)
                if (!(fl[k - 1] & kHugeTerm) && E[k - 1] != kHugeNone && S[k] != E[k - 1]) from[k] = E[k - 1], any = true;
            if (!any || guard > (int)P + 2) break;
            for (uint32_t k = 1; k < P; ++k)
                if (from[k] != kHugeNone) {
                    huge_refix<2>(ld16, T.lut2, T.lo, in_mis, nb, k, P, PB, from[k], S[k], E[k], c[k], fl[k]);
                    ++*fixes;
                }
        }
        uint32_t t = kHugeNone;
        for (uint32_t k = 0; k < P && t == kHugeNone; ++k)
            if (fl[k] & kHugeTerm) t = k;
        if (t == kHugeNone) {
            printf("huge: no terminal piece (%u B)\n", nb);
            ++bad;
            continue;
        }
        uint32_t D = 0;
        for (uint32_t k = 0; k <= t; ++k) {
            huge_pass2<2>(ld16, T.lut2, T.lo, in_mis, S[k], c[k], out_mis + D, st8, st1);
            D += c[k];
        }
        const uint32_t olen = D, ost = fl[t] & 0xFFu;
        std::vector<uint8_t> ref(cap + 8);
        size_t rl = 0;
        const int rs = oracle_decode(enc.data(), nb, ref.data(), ref.size(), &rl);
        const bool ok = rs == (int)ost && rl == olen && memcmp(ref.data(), out_base + out_mis, rl) == 0;
        if (!ok && bad < 5)
            printf("huge: literal of %u B kind %d (P %u, PB %u): status %u vs %d, length %u vs %zu\n", nb, kind, P, PB, ost, rs,
                   olen, rl);
        bad += !ok;
        for (uint32_t j = 0; j < outb.size(); ++j)
            if ((j < 16 + out_mis || j >= 16 + out_mis + std::max<uint32_t>(olen, 0)) && j >= 16 + out_mis + cap &&
                outb[j] != 0xEE) {
                if (bad < 5) printf("huge: guard byte %u written (%u B)\n", j, nb);
                ++bad;
                break;
            }
        for (uint32_t j = 0; j < 16 + out_mis; ++j)
            if (outb[j] != 0xEE) {
                if (bad < 5) printf("huge: byte before the region written (%u B)\n", nb);
                ++bad;
                break;
            }
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
    }
    long fixes = 0;
    bad += run_huge(rng, iters * 3, 1024, &fixes);
    bad += run_huge(rng, iters, 64, &fixes);
    printf("huge: %ld pieces walked again\n", fixes);
    printf("%s: %d mismatches\n", bad ? "FAIL" : "ok", bad);
    return bad != 0;
}
