// hpk_persist.h — the small-call mode (hpk_ctx_set_small_mode, round 6): a persistent decode kernel
// with its tables resident in LDS that takes synchronous device-pointer batches through a host-mapped
// doorbell, so a small call skips the kernel launch (~4 us of API, ~5 us to the kernel's start) and
// the stream synchronisation (~5 us from the kernel's end to the host's wake-up) of the launch path
// (DESIGN.md §6). One lane per literal, walking its input straight from global memory with the
// two-symbol table (the huge phase's walker, hpk_huge.h) and storing whole 8-byte groups.
//
// Protocol (PersistCtl lives in host memory, coherent and mapped; the host writes a request's
// fields, then req; the device answers with done = req):
//   * workgroup 0's first wave polls req / stop (relaxed system-scope loads, no fence per poll),
//     reads the request's fields one per lane and broadcasts them and the command, or the exit,
//     through device memory; the other workgroups poll that (relaxed agent-scope loads);
//   * every workgroup decodes literals wg * kThreads + tid, wg * kThreads + tid + G * kThreads, ...;
//     a literal with bad offsets is not decoded and marks the request declined (the host then runs
//     it through the launch path, which writes the ABI's HPK_BAD_OFFSETS results);
//   * each workgroup takes one agent-scope acquire per request, and counts itself after one
//     agent-scope release; the last one of the request publishes declined and done to the host;
//   * exits every wave reaches: workgroup 0 broadcasts the exit when the host sets stop or when no
//     request came for idle_ticks of the 100 MHz real-time clock, and clears alive; the other
//     workgroups also leave on their own after 8 x idle_ticks without a command (a safety net only:
//     workgroup 0 always broadcasts first). Nothing loops on a value only the host could change
//     without a deadline.
#pragma once

namespace hpkdec {

struct PersistCtl {  // host memory (hipHostMallocMapped | hipHostMallocCoherent), one cache line apart
    uint32_t req;       // host: the last request number issued
    uint32_t stop;      // host: 1 = exit now
    uint32_t pad0[14];
    uint32_t done;      // device: the last request finished
    uint32_t declined;  // device: the last finished request was not decoded (bad offsets)
    uint32_t alive;     // host sets 1 at launch; device clears it when it exits
    uint32_t ts[6];     // device: 100 MHz stamps of the last request (hpk_test_small_stamps): workgroup 0 saw it,
                        // broadcast it, finished its literals; the last workgroup published it; then workgroup 0's
                        // shader-clock cycles between the broadcast and its finish, and the same in 100 MHz ticks
    uint32_t tl[4];     // device: thread 0's first literal of the last request, shader-clock cycles from the
                        // command to the offsets loaded, to the literal staged, to its walk done, to its stores issued
    uint32_t pad1[3];
    // the request (written by the host before req)
    const uint8_t* in_base;
    uint8_t* out_base;
    const uint32_t* in_off;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
    uint32_t n, in_mis, out_mis, in_cap, out_cap, pad2[3];
};

struct PersistArgs {
    PersistCtl* ctl;  // device-visible pointer to the host block
    uint32_t* dev;    // [0] workgroups finished since launch, [1] cmd broadcast, [2] declined flag (request number),
                      // [4, 21) the request's fields (workgroup 0's copy)
    const uint32_t* lut3;
    const uint16_t* lo;
    uint32_t base;        // requests up to this number were finished before the launch
    uint32_t idle_ticks;  // 100 MHz ticks without a request before the kernel exits
};

constexpr uint32_t kPersistExit = 0xFFFFFFFFu;

// The request's pointers come from memory, not from kernel arguments, so the compiler cannot tell they are
// global and would use flat accesses, which count in lgkmcnt too: every LDS lookup of the walk then waited
// for the output stores in flight (~27 us for one 27-byte literal per lane). Global address space, explicitly.
#define HPK_GAS __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ HPK_GAS T* gas(T* p) {
    return (HPK_GAS T*)p;
}

#ifndef HPK_PERSIST_SLEEP
#define HPK_PERSIST_SLEEP 2  // s_sleep between polls (units of 64 cycles)
#endif

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One literal: huffman.rs:95-161 semantics (a code that runs past the end ends the walk, EOS is
// EOSInString at once, then > 7 residual bits PaddingTooLarge, non-ones InvalidPadding), and the batch
// ABI's capacity check per byte (HPK_OUTPUT_OVERFLOW, as the fill kernels' byte path:
// hpk_decode_kernel.h lit_bytes_to). Returns false (nothing written) if the literal's offsets are bad.
template <class Ld>
__device__ bool persist_literal(const Ld& ld16, const uint32_t* __restrict__ lut, const uint16_t* __restrict__ lo,
                                HPK_GAS uint8_t* out_base, uint32_t out_mis, uint32_t in_mis, uint32_t p0, uint32_t p1,
                                uint32_t o0, uint32_t o1, uint32_t& cnt, uint32_t& st) {
    const uint32_t nbits = (p1 - p0) * 8u, cap = o1 - o0;
    const uint32_t ob = out_mis + o0;  // (out_base-relative)
    cnt = 0;
    st = HPK_OK;
    if (nbits == 0u) return true;
    HugeWalk W;
    huge_begin(W, ld16, p0 + in_mis, 0u);
    uint64_t acc = 0;  // pending bytes of the 8-byte group holding position ob + cnt
    auto emit = [&](uint32_t sym) {
        const uint32_t p = ob + cnt;
        acc |= (uint64_t)sym << (8u * (p & 7u));
        if ((p & 7u) == 7u) {  // a group is complete: 8 bytes at once, or its bytes from ob on
            const uint32_t g = p - 7u;
            if (g >= ob)
                *(HPK_GAS uint64_t*)(out_base + g) = acc;
            else
                for (uint32_t x = ob; x <= p; ++x) out_base[x] = (uint8_t)(acc >> (8u * (x & 7u)));
            acc = 0;
        }
        cnt += 1u;
    };
    while (W.pos < nbits) {
        uint32_t sym, len, sym1, held;
        bool eos;
        huge_peek<3>(W, ld16, lut, lo, sym, len, eos, sym1, held);
        const uint32_t rem = nbits - W.pos;
        if (held != 0u && held <= rem && cnt + 2u <= cap) {  // two codes of <= 12 bits, both inside
            emit(sym);
            emit(sym1);
            huge_adv(W, held);
            continue;
        }
        if (len > rem) {  // huffman.rs:128-160
            st = residual_status(rem, (uint32_t)(W.win >> 32));
            break;
        }
        if (eos) {  // huffman.rs:112-116
            st = HPK_EOS_IN_STRING;
            break;
        }
        if (cnt >= cap) {
            st = HPK_OUTPUT_OVERFLOW;
            break;
        }
        emit(sym);
        huge_adv(W, len);
    }
    const uint32_t pe = ob + cnt;  // the last partial group, bytewise
    for (uint32_t x = max(ob, pe & ~7u); x < pe; ++x) out_base[x] = (uint8_t)(acc >> (8u * (x & 7u)));
    return true;
}

// The same walk over the literal staged in LDS: its 16-byte chunks loaded at once (one memory latency
// instead of one per chunk crossing: the global walker above took ~30 us for a 27-byte literal), stored
// big-endian into the lane's slot (dword j of lane t at slot[j * kThreads + t]: no bank conflicts).
constexpr uint32_t kPersistSlotChunks = 8;  // 128 bytes per lane: literals of <= 113 bytes (else the global walk)
constexpr uint32_t kPersistSlotMax = 113;   // (their decoded bound, 180 bytes, fits the output slot)

// Output: the walk writes the literal's bytes into the lane's LDS output slot, at the byte's position on
// the global 4-byte grid (slot byte (ob & 3) + k), and they leave it after the walk: the head's bytes up
// to the first 4-aligned address, then every whole dword, then the tail's bytes, the stores unrolled with
// their own registers. (Stores inside the walk made it wait for each one to complete before the next
// group's register could be written: ~25 us for a 27-byte literal.)
constexpr uint32_t kPersistOutDw = 48;  // output slot dwords per lane: 113 bytes decode to <= 180, + 3 of alignment, + 4
                                        // of a body step's garbage; the last byte is the checked steps' dummy

// Input slot: the lane's chunks as contiguous big-endian dwords after one pad dword (the lane walk reads
// dword (X >> 5) - 1), lane t's at slot + t * kPersistInStride: an odd stride, so the lanes' reads of the
// same dword fall in different banks.
constexpr uint32_t kPersistInStride = 4u * kPersistSlotChunks + 1u;

template <int kThreads>
__device__ void persist_literal_lds(const HPK_GAS u32x4* __restrict__ g16, uint32_t last16, uint32_t* __restrict__ win32,
                                    uint8_t* __restrict__ oslot, const uint32_t* __restrict__ lut,
                                    const uint16_t* __restrict__ lo, HPK_GAS uint8_t* out_base, uint32_t out_mis,
                                    uint32_t in_mis, uint32_t p0, uint32_t p1, uint32_t o0, uint32_t o1, uint32_t& cnt,
                                    uint32_t& st, uint64_t* tl = nullptr) {
    const uint32_t nbytes = p1 - p0, b0 = p0 + in_mis, nbits = nbytes * 8u, cap = o1 - o0;
    const uint32_t c0 = b0 >> 4, nch = ((b0 + nbytes + 15u) >> 4) - c0;  // (<= kPersistSlotChunks)
    const uint32_t ob = out_mis + o0;
    const uint32_t oa = ob & 3u;  // the output slot's first byte sits at its global address mod 4
    cnt = 0;
    st = HPK_OK;
    if (nbits == 0u) return;
    u32x4 v[kPersistSlotChunks];
#pragma unroll
    for (uint32_t j = 0; j < kPersistSlotChunks; ++j) v[j] = j < nch ? g16[min(c0 + j, last16)] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t j = 0; j < kPersistSlotChunks; ++j) {
        win32[1u + 4u * j] = hpk_bswap32(v[j].x);
        win32[2u + 4u * j] = hpk_bswap32(v[j].y);
        win32[3u + 4u * j] = hpk_bswap32(v[j].z);
        win32[4u + 4u * j] = hpk_bswap32(v[j].w);
    }
    if (tl) tl[1] = __builtin_amdgcn_s_memtime();
    const uint32_t sb = 32u + (b0 & 15u) * 8u;  // the literal's first bit in the window
    if (cap >= (nbytes * 8u) / 5u) {
        // a region that holds the decoded bound: the wave kernel's lane walk (body steps while >= kBodyMin
        // bits are left, then checked steps), bytes into the output slot, unconditional stores (kPred:
        // the dummy byte at kPersistOutDw * 4 - 1)
        Lit12 L;
        L.X = sb + 31u;
        L.Eb = L.X + nbits;
        L.o = oa;
        L.o0 = oa;
        L.oend = 0;
        L.st = HPK_OK;
        L.more = true;
        lit12_load(L, win32);
        bool body = L.Eb - L.X >= kBodyMin;
        while (body) lit12_body<kPred, 3>(L, win32, lut, lo, oslot, body);
        while (L.more) lit12_step<kPred, false, 3, true>(L, win32, lut, lo, oslot, kPersistOutDw * 4u - 1u);
        cnt = L.o - L.o0;
        st = lit12_status(L);
    } else {
        // a region below the decoded bound: code by code, the capacity checked per byte (the fill kernels'
        // byte path, hpk_decode_kernel.h lit_bytes_to)
        uint32_t q = sb >> 5;
        uint64_t win = ((uint64_t)win32[q] << 32) << (sb & 31u);
        uint32_t nb = 32u - (sb & 31u), pos = 0;
        q += 1u;
        while (pos < nbits) {
            if (nb <= 32u) {  // (q stays inside the slot: past the literal's chunks it reads zeros)
                win |= (uint64_t)win32[min(q, 4u * kPersistSlotChunks)] << (32u - nb);
                nb += 32u;
                q += 1u;
            }
            const uint32_t w = (uint32_t)(win >> 32);
            uint32_t sym, len;
            bool eos;
            lo_decode(w, lo, sym, len, eos);
            const uint32_t rem = nbits - pos;
            if (len > rem) {  // huffman.rs:128-160
                st = residual_status(rem, w);
                break;
            }
            if (eos) {  // huffman.rs:112-116
                st = HPK_EOS_IN_STRING;
                break;
            }
            if (cnt >= cap) {
                st = HPK_OUTPUT_OVERFLOW;
                break;
            }
            oslot[oa + cnt] = (uint8_t)sym;
            cnt += 1u;
            win <<= len;
            nb -= len;
            pos += len;
        }
    }
    if (tl) tl[2] = __builtin_amdgcn_s_memtime();
    // [ob, ob + cnt): head bytes up to the 4-aligned address h, whole dwords [h, t), tail bytes [t, ob + cnt)
    const uint32_t e = ob + cnt, h = min((ob + 3u) & ~3u, e), t = max(e & ~3u, h);
#pragma unroll
    for (uint32_t k = 0; k < 3u; ++k)
        if (ob + k < h) out_base[ob + k] = oslot[oa + k];
    // the dwords: those before the first 16-aligned address h16 and from the last one t16 on singly, the
    // 16-byte groups between as 16-byte stores (a store instruction per group, not per dword)
    const uint32_t* const os32 = reinterpret_cast<const uint32_t*>(oslot);
    const uint32_t base = ob - oa;  // the slot's first byte's address (4-aligned)
    const uint32_t h16 = min((h + 15u) & ~15u, t), t16 = max(t & ~15u, h16);
#pragma unroll
    for (uint32_t k = 0; k < 3u; ++k)
        if (h + 4u * k < h16) *reinterpret_cast<HPK_GAS uint32_t*>(out_base + h + 4u * k) = os32[(h - base) / 4u + k];
#pragma unroll
    for (uint32_t k = 0; k < kPersistOutDw / 4u; ++k)
        if (h16 + 16u * k < t16) {
            const uint32_t d = (h16 - base) / 4u + 4u * k;
            *reinterpret_cast<HPK_GAS u32x4*>(out_base + h16 + 16u * k) = u32x4{os32[d], os32[d + 1u], os32[d + 2u], os32[d + 3u]};
        }
#pragma unroll
    for (uint32_t k = 0; k < 3u; ++k)
        if (t16 + 4u * k < t) *reinterpret_cast<HPK_GAS uint32_t*>(out_base + t16 + 4u * k) = os32[(t16 - base) / 4u + k];
#pragma unroll
    for (uint32_t k = 0; k < 3u; ++k)
        if (t + k < e) out_base[t + k] = oslot[t + k - (ob - oa)];
    if (tl) tl[3] = __builtin_amdgcn_s_memtime();
}

template <int kThreads>
__global__ __launch_bounds__(kThreads) void hpk_persist(PersistArgs p) {
    // Memory model (MI355X: one L2 per XCD, not coherent with the others). Polling uses relaxed loads
    // that bypass the caches (no fence per poll: an acquire at agent or system scope invalidates the
    // XCD's L2, which a poll loop would do continuously, for every kernel on that XCD). Per request each
    // workgroup takes ONE acquire after it has seen the command (the input was written by kernels that
    // finished before the call, maybe on another XCD) and ONE release before it counts itself.
    __shared__ uint32_t s_lut[HPK_LUT_SIZE];
    __shared__ uint16_t s_lo[HPK_LO_SIZE];
    __shared__ uint32_t s_cmd[18];
    __shared__ uint32_t s_slot[kPersistInStride * kThreads];  // per lane: its literal's input (staged)
    __shared__ uint32_t s_oslot[kPersistOutDw * kThreads];          // per lane: its literal's output
    const uint32_t tid = threadIdx.x, lane = tid & 63u, G = gridDim.x, wg = blockIdx.x;
    for (uint32_t t = tid; t < (uint32_t)HPK_LUT_SIZE; t += kThreads) s_lut[t] = p.lut3[t];
    for (uint32_t t = tid; t < (uint32_t)HPK_LO_SIZE; t += kThreads) s_lo[t] = p.lo[t];
    PersistCtl* const ctl = p.ctl;
    uint32_t* const fields = p.dev + 4;  // (device copy of the request's 17 dwords, made by workgroup 0)
    uint32_t seen = p.base;
    uint32_t served = 0;  // requests this launch finished (the count's target)
    uint64_t t_bc = 0, r_bc = 0;  // (workgroup 0, thread 0) clocks at the broadcast
    for (;;) {
        if (tid < 64u) {  // wave 0: wait for the next command
            uint32_t cmd = kPersistExit;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            if (wg == 0) {  // the doorbell (lane 0's loads; the wave follows it)
                for (;;) {
                    uint32_t r = 0, stop = 0;
                    if (lane == 0) {
                        r = __hip_atomic_load(&ctl->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        stop = __hip_atomic_load(&ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
                    stop = (uint32_t)__builtin_amdgcn_readfirstlane((int)stop);
                    if (r != seen) {
                        cmd = r;
                        if (lane == 0) ctl->ts[0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                        break;
                    }
                    if (stop != 0u) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)p.idle_ticks) break;
                    __builtin_amdgcn_s_sleep(HPK_PERSIST_SLEEP);
                }
                if (cmd != kPersistExit) {  // the request's fields (the host wrote them before req), one per lane
                    if (lane < 17u) {
                        const uint32_t* f = reinterpret_cast<const uint32_t*>(&ctl->in_base);
                        const uint32_t v = __hip_atomic_load(f + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        s_cmd[1 + lane] = v;
                        fields[lane] = v;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // (the fields before the command)
                if (lane == 0) {
                    __hip_atomic_store(&p.dev[1], cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ctl->ts[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                }
                t_bc = __builtin_amdgcn_s_memtime();
                r_bc = __builtin_amdgcn_s_memrealtime();
            } else {  // workgroup 0's broadcast
                for (;;) {
                    uint32_t r = 0;
                    if (lane == 0) r = __hip_atomic_load(&p.dev[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
                    if (r != seen) {
                        cmd = r;
                        break;
                    }
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 8ull * p.idle_ticks) break;  // (safety net)
                    __builtin_amdgcn_s_sleep(HPK_PERSIST_SLEEP);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                if (cmd != kPersistExit && lane < 17u) s_cmd[1 + lane] = fields[lane];
            }
            if (lane == 0) s_cmd[0] = cmd;
        }
        __syncthreads();
        const uint32_t cmd = s_cmd[0];
        if (cmd == kPersistExit) break;
        // the input and the offsets were written by kernels that finished before the call: one acquire
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        auto ptr = [&](int k) { return ((uint64_t)s_cmd[k + 1] << 32) | s_cmd[k]; };
        const HPK_GAS uint8_t* in_base = gas(reinterpret_cast<const uint8_t*>(ptr(1)));
        HPK_GAS uint8_t* out_base = gas(reinterpret_cast<uint8_t*>(ptr(3)));
        const HPK_GAS uint32_t* in_off = gas(reinterpret_cast<const uint32_t*>(ptr(5)));
        const HPK_GAS uint32_t* out_off = gas(reinterpret_cast<const uint32_t*>(ptr(7)));
        HPK_GAS uint32_t* out_len = gas(reinterpret_cast<uint32_t*>(ptr(9)));
        HPK_GAS uint8_t* status = gas(reinterpret_cast<uint8_t*>(ptr(11)));
        const uint32_t n = s_cmd[13], in_mis = s_cmd[14], out_mis = s_cmd[15], in_cap = s_cmd[16], out_cap = s_cmd[17];
        __syncthreads();  // (every thread has read s_cmd before wave 0 writes the next command)
        const uint32_t in_end = (n ? min(in_off[n], in_cap) : 0u) + in_mis;
        const uint32_t last16 = in_end ? (in_end - 1u) >> 4 : 0u;
        const HPK_GAS u32x4* const g16 = reinterpret_cast<const HPK_GAS u32x4*>(in_base);
        auto ld16 = [&](uint32_t ci) {
            const u32x4 v = g16[min(ci, last16)];
            return make_uint4(v.x, v.y, v.z, v.w);
        };
        bool bad = false;
        uint64_t tlv[4] = {0, 0, 0, 0};
        const uint64_t tcmd = __builtin_amdgcn_s_memtime();
        for (uint32_t i = wg * kThreads + tid; i < n; i += G * kThreads) {
            const uint32_t p0 = in_off[i], p1 = in_off[i + 1], o0 = out_off[i], o1 = out_off[i + 1];
            if (i == 0u) tlv[0] = __builtin_amdgcn_s_memtime() + (uint64_t)(p0 & 0u);
            if (!(p0 <= p1 && p1 <= in_cap && o0 <= o1 && o1 <= out_cap)) {
                bad = true;
                continue;
            }
            uint32_t cnt, st;
            const uint32_t b0 = p0 + in_mis;
            if (((b0 + (p1 - p0) + 15u) >> 4) - (b0 >> 4) <= kPersistSlotChunks && p1 - p0 <= kPersistSlotMax)
                persist_literal_lds<kThreads>(g16, last16, s_slot + kPersistInStride * tid,
                                              reinterpret_cast<uint8_t*>(s_oslot + kPersistOutDw * tid), s_lut, s_lo,
                                              out_base, out_mis, in_mis, p0, p1, o0, o1, cnt, st, i == 0u ? tlv : nullptr);
            else  // (a longer literal: walked from global memory)
                persist_literal(ld16, s_lut, s_lo, out_base, out_mis, in_mis, p0, p1, o0, o1, cnt, st);
            out_len[i] = cnt;
            status[i] = (uint8_t)st;
        }
        if (wg == 0 && tid == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) ctl->tl[k] = (uint32_t)(tlv[k] - (k ? tlv[k - 1] : tcmd));
        }
        if (bad) __hip_atomic_store(&p.dev[2], cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        served += 1u;
        __syncthreads();  // (the workgroup's stores are in its L2: a workgroup-scope release waits for them)
        if (tid == 0) {
            if (wg == 0) {
                const uint64_t r2 = __builtin_amdgcn_s_memrealtime(), t2 = __builtin_amdgcn_s_memtime();
                ctl->ts[2] = (uint32_t)r2;
                ctl->ts[4] = (uint32_t)(t2 - t_bc);
                ctl->ts[5] = (uint32_t)(r2 - r_bc);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the workgroup's results to memory, once
            const uint32_t prev = __hip_atomic_fetch_add(&p.dev[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev + 1u == served * G) {  // the request's last workgroup: publish it to the host
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                const uint32_t dec = __hip_atomic_load(&p.dev[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == cmd;
                __hip_atomic_store(&ctl->declined, dec ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                ctl->ts[3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                st_sys(&ctl->done, cmd);
            }
        }
        seen = cmd;
    }
    if (wg == 0 && tid == 0) st_sys(&ctl->alive, 0u);
}

}  // namespace hpkdec
