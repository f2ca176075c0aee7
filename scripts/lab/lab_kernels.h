// lab_kernels.h -- candidate C2 decode kernels (development only).
#pragma once

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

struct DescOutL {
    uint32_t key_off, key_len, val_off, val_len;
    uint64_t trailer;
    uint32_t file_num, fnv1, crc, status;
};
__device__ __forceinline__ void store_descL(bhg_desc *out, const DescOutL &d) {
    uint2 *o = reinterpret_cast<uint2 *>(out);
    o[0] = make_uint2(d.key_off, d.key_len);
    o[1] = make_uint2(d.val_off, d.val_len);
    o[2] = make_uint2((uint32_t)d.trailer, (uint32_t)(d.trailer >> 32));
    o[3] = make_uint2(d.file_num, d.fnv1);
    o[4] = make_uint2(d.crc, d.status);
}

struct PrefixL {
    uint32_t rw[15];
    __device__ __forceinline__ void load(uint64_t p, uint64_t end) {
        const uint64_t a = p & ~3ull;
        const uint32_t sh = (uint32_t)(p & 3);
        uint32_t w[16];
        if (a + 64 <= end) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 v = gld<u32x4_a4>(a + 16 * q);
                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = ld32_safe(a + 4 * j, end);
        }
#pragma unroll
        for (int j = 0; j < 15; j++) rw[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
    }
    __device__ __forceinline__ uint32_t word_at(uint32_t byte) const {
        const uint32_t t = byte >> 2, s = byte & 3;
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (uint32_t j = 3; j < 14; j++) {
            lo = t == j ? rw[j] : lo;
            hi = t == j ? rw[j + 1] : hi;
        }
        return __builtin_amdgcn_alignbyte(hi, lo, s);
    }
    __device__ __forceinline__ uint32_t fnv_key(uint32_t klen) const {
        uint32_t h = BHG_FNV_OFFSET;
        const uint32_t stop = 12 + klen;
#pragma unroll
        for (uint32_t j = 3; j < 15; j++) {
            if (4 * j >= stop) break;
#pragma unroll
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t hn = (h * BHG_FNV_PRIME) ^ ((rw[j] >> (8 * b)) & 0xffu);
                h = 4 * j + b < stop ? hn : h;
            }
        }
        return h;
    }
};

// header / key / trailer / FNV-1 from the prefix registers (readRecord + readKV)
struct RecHead {
    uint32_t k, v, fn, key_len, fnv;
    uint64_t trailer;
    bool valid;
    __device__ __forceinline__ void parse(uint64_t p, uint32_t L, uint64_t end) {
        PrefixL P;
        P.load(p, end);
        k = L >= 12 ? P.rw[0] : 0;
        v = L >= 12 ? P.rw[1] : 0;
        fn = P.rw[2];
        valid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
        key_len = 0;
        fnv = BHG_FNV_OFFSET;
        trailer = 255;
        if (valid && k >= 8) {
            key_len = k - 8;
            if (key_len <= 36) {
                fnv = P.fnv_key(key_len);
                trailer = (uint64_t)P.word_at(12 + key_len) | ((uint64_t)P.word_at(16 + key_len) << 32);
            } else {
                fnv = fnv1_range(p + 12, key_len, end);
                trailer = ldu64(p + 12 + k - 8, end);
            }
        }
    }
    __device__ __forceinline__ DescOutL desc(uint32_t crc) const {
        if (!valid) return DescOutL{0, 0, 0, 0, 0, 0, 0, crc, BHG_ST_RECORD_NIL};
        return DescOutL{12, key_len, 12 + k, v, trailer, fn, fnv, crc, BHG_ST_OK};
    }
};

// ============================================================== E1: per-lane, perm table
template <int WG, int WIN>
__global__ __launch_bounds__(WG) void k_lane_perm(const uint8_t *__restrict__ src, uint64_t src_len,
                                                  const bhg_handle *__restrict__ handles, uint32_t n,
                                                  bhg_desc *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    Crc4Perm::fill(T);
    __syncthreads();
    const Crc4Perm crc(T);
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bhg_handle hn = {0, 0, 0};
    if (i < n) hn = handles[i];
    for (; i < n; i += stride) {
        const bhg_handle h = hn;
        if (i + stride < n) hn = handles[i + stride];
        DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, BHG_ST_OK};
        if (h.length == 0) {
            d.status = BHG_ST_ILLEGAL_LENGTH;
        } else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) {
            d.status = BHG_ST_INCOMPLETE;
        } else {
            const uint64_t p = base + h.offset;
            RecHead H;
            H.parse(p, h.length, end);
            const uint32_t c = crc_mask(~crc_range_a<WIN, Crc4Perm, true>(crc, 0xffffffffu, p, h.length, end));
            d = H.desc(c);
        }
        store_descL(out + i, d);
    }
}


// ============================================================== E4: per-lane walk, shared lines loaded together
// Lane per record.  The record's head line (p & ~127) and tail line
// ((E-1) & ~127) are loaded first, in the same instructions as the
// neighbouring lanes' tail/head lines (the same physical line), and the tail
// line is held in registers until the interior lines -- owned by this lane
// alone -- have been absorbed.  Every line is then fetched once.
__device__ __forceinline__ void load_line(u32x4 *v, uint64_t a, uint64_t lo, uint64_t hi) {
    if (a >= lo && a + 128 <= hi) {
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = gld<u32x4>(a + 16 * q);
    } else {
#pragma unroll
        for (int q = 0; q < 8; q++) {
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t x = a + 16 * q + 4 * k;
                w[k] = (x >= lo && x + 4 <= hi) ? gld<uint32_t>(x) : ((x >= lo && x < hi) ? ld32_safe(x, hi) : 0u);
            }
            v[q] = u32x4{w[0], w[1], w[2], w[3]};
        }
    }
}
__device__ __forceinline__ uint32_t lw(const u32x4 *v, int t) {
    return t % 4 == 0 ? v[t / 4].x : t % 4 == 1 ? v[t / 4].y : t % 4 == 2 ? v[t / 4].z : v[t / 4].w;
}
// absorb bytes [b0, b1) (0 <= b0 <= b1 <= 128) of a line held in v
template <class Tab>
__device__ __forceinline__ uint32_t absorb_line(const Tab &T, uint32_t c, const u32x4 *v, uint32_t b0, uint32_t b1) {
    const uint32_t t0 = (b0 + 3) >> 2, t1 = b1 >> 2;  // full words [t0, t1)
    if (b0 & 3) {  // head partial word
        const uint32_t tw = b0 >> 2;
        uint32_t x = 0;
#pragma unroll
        for (int t = 0; t < 32; t++) x = (uint32_t)t == tw ? lw(v, t) : x;
        const uint32_t nb = (tw == (b1 >> 2)) ? (b1 - b0) : (4 - (b0 & 3));
        c = T.partial(c, x >> (8 * (b0 & 3)), nb);
        if (tw == (b1 >> 2)) return c;
    }
#pragma unroll
    for (int t = 0; t < 32; t++)
        if ((uint32_t)t >= t0 && (uint32_t)t < t1) c = T.word(c, lw(v, t));
    if ((b1 & 3) && t1 >= t0) {  // tail partial word
        uint32_t x = 0;
#pragma unroll
        for (int t = 0; t < 32; t++) x = (uint32_t)t == t1 ? lw(v, t) : x;
        c = T.partial(c, x, b1 & 3);
    }
    return c;
}
template <int WG, int MODE>
__global__ __launch_bounds__(WG) void k_lane3(const uint8_t *__restrict__ src, uint64_t src_len,
                                              const bhg_handle *__restrict__ handles, uint32_t n,
                                              bhg_desc *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    Crc4Perm::fill(T);
    __syncthreads();
    const Crc4Perm crc(T);
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const bhg_handle h = handles[i];
        DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, BHG_ST_OK};
        if (h.length == 0) {
            d.status = BHG_ST_ILLEGAL_LENGTH;
        } else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) {
            d.status = BHG_ST_INCOMPLETE;
        } else {
            const uint64_t p = base + h.offset, e = p + h.length;
            const uint64_t ha = p & ~127ull, ta = (e - 1) & ~127ull;
            u32x4 H[8], Tl[8];
            load_line(H, ha, base, end);
            if (ta != ha) load_line(Tl, ta, base, end);
            RecHead R;
            R.parse(p, h.length, end);
            uint32_t c = 0xffffffffu;
            if (MODE == 1) {
#pragma unroll
                for (int t = 0; t < 32; t++) c ^= lw(H, t);
            } else {
                c = absorb_line(crc, c, H, (uint32_t)(p - ha), ta == ha ? (uint32_t)(e - ha) : 128u);
            }
            if (ta != ha) {
                // interior lines, one window in flight ahead
                u32x4 A[8], B[8];
                uint64_t w = ha + 128;
                if (w < ta) load_line(A, w, base, end);
                while (w < ta) {
                    const uint64_t w1 = w + 128;
                    if (w1 < ta) load_line(B, w1, base, end);
                    if (MODE == 1) {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = ((c << 1) | (c >> 31)) ^ lw(A, t);
                    } else {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = crc.word(c, lw(A, t));
                    }
                    if (w1 >= ta) break;
                    const uint64_t w2 = w1 + 128;
                    if (w2 < ta) load_line(A, w2, base, end);
                    if (MODE == 1) {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = ((c << 1) | (c >> 31)) ^ lw(B, t);
                    } else {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = crc.word(c, lw(B, t));
                    }
                    w = w2;
                }
                if (MODE == 1) {
#pragma unroll
                    for (int t = 0; t < 32; t++) c ^= lw(Tl, t);
                } else {
                    c = absorb_line(crc, c, Tl, 0u, (uint32_t)(e - ta));
                }
            }
            d = R.desc(crc_mask(~c));
        }
        store_descL(out + i, d);
    }
}


// ============================================================== E5: dense sweep of small record rounds
// Round = RPR consecutive whole records; wave w takes rounds w, w+W, ... so the
// chip reads one dense region at a time.  Each record is cut into 128 B
// chunks aligned to its END (chunk 0 = head, 1..128 B); one chunk per lane
// (passes of 64 chunks).  Lane: CRC of its chunk (head chunk from
// 0xFFFFFFFF, others from 0) -> LDS; record lane: Horner fold
// S = Z128(S) ^ V_q over its chunks.
template <int WAVES, int MODE>
__global__ __launch_bounds__(64 * WAVES) void k_sweep(const uint8_t *__restrict__ src, uint64_t src_len,
                                                      const bhg_handle *__restrict__ handles, uint32_t n,
                                                      bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz128,
                                                      uint32_t rpr) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[1024];
    __shared__ uint32_t V[WAVES][64];
    Crc4Perm::fill(T);
    for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) Z[t] = gz128[t];
    __syncthreads();
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t nrounds = (n + rpr - 1) / rpr;
    const uint32_t W = gridDim.x * WAVES;
    uint32_t round = blockIdx.x * WAVES + wave;
    bhg_handle hn = {0, 0, 0};
    if (round < nrounds && lane < rpr && round * rpr + lane < n) hn = handles[round * rpr + lane];
    for (; round < nrounds; round += W) {
        const uint32_t i = round * rpr + lane;
        const bool mine = lane < rpr && i < n;
        const bhg_handle h = hn;
        {
            const uint32_t nr = round + W;
            hn = bhg_handle{0, 0, 0};
            if (nr < nrounds && lane < rpr && nr * rpr + lane < n) hn = handles[nr * rpr + lane];
        }
        bool inb = false;
        uint32_t st = BHG_ST_OK;
        if (mine) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint64_t p = base + h.offset;
        const uint32_t L = inb ? h.length : 0u;
        const uint32_t m = inb ? (L + 127) >> 7 : 0u;
        uint32_t incl = m;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += t;
        }
        const uint32_t cs = incl - m;
        const uint32_t M = __shfl(incl, 63, 64);
        uint32_t S = 0;
        for (uint32_t pb = 0; pb < M; pb += 64) {
            const uint32_t c = pb + lane;
            uint32_t r = 0;
            for (uint32_t j = 1; j < rpr; j++) r += (uint32_t)__shfl(cs, j, 64) <= c ? 1u : 0u;
            const uint64_t pr = shfl64(p, r);
            const uint32_t Lr = __shfl(L, r, 64), mr = __shfl(m, r, 64), csr = __shfl(cs, r, 64);
            const uint32_t q = c - csr;
            const uint32_t hs = Lr - 128u * (mr - 1);
            const uint64_t cst = pr + (q ? hs + 128u * (q - 1) : 0u);
            const uint32_t clen = c < M ? (q ? 128u : hs) : 0u;
            uint32_t v = q == 0 ? 0xffffffffu : 0u;
            if (clen) {
                const uint64_t a0 = cst & ~3ull;
                const uint32_t sh = (uint32_t)(cst & 3);
                uint32_t w[33];
                if (a0 + 132 <= end) {
#pragma unroll
                    for (uint32_t qq = 0; qq < 8; qq++) {
                        const u32x4 x = gld<u32x4_a4>(a0 + 16 * qq);
                        w[4 * qq] = x.x; w[4 * qq + 1] = x.y; w[4 * qq + 2] = x.z; w[4 * qq + 3] = x.w;
                    }
                    w[32] = gld<uint32_t>(a0 + 128);
                } else {
#pragma unroll
                    for (uint32_t t = 0; t <= 32; t++) w[t] = ld32_safe(a0 + 4 * t, end);
                }
                const uint32_t nw = clen >> 2, tail = clen & 3;
                if (MODE == 1) {
#pragma unroll
                    for (uint32_t t = 0; t < 32; t++)
                        if (t < nw) v = ((v << 1) | (v >> 31)) ^ __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                } else {
#pragma unroll
                    for (uint32_t t = 0; t < 32; t++)
                        if (t < nw) v = crc.word(v, __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh));
                }
                if (tail) v = crc.partial(v, ldu32(cst + 4 * nw, end), tail);
            }
            V[wave][lane] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (m) {
                const uint32_t q0 = pb > cs ? pb - cs : 0u;
                const uint32_t q1 = min(m, pb + 64 - cs);
                for (uint32_t qq = q0; qq < q1 && cs + qq >= pb; qq++) {
                    const uint32_t x = V[wave][cs + qq - pb];
                    if (MODE == 1) S = ((S << 1) | (S >> 31)) ^ x;
                    else S = (qq == 0 ? 0u : (Z[S & 255u] ^ Z[256 + ((S >> 8) & 255u)] ^ Z[512 + ((S >> 16) & 255u)] ^ Z[768 + (S >> 24)])) ^ x;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        RecHead H;
        if (inb) H.parse(p, L, end);
        if (mine) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) d = H.desc(crc_mask(~S));
            store_descL(out + i, d);
        }
    }
}


// ============================================================== E6: pipelined dense sweep
struct SwRound {
    // record lane (lane < rpr)
    uint64_t p;
    uint32_t L, m, cs, st, M;
    bool mine, inb;
    // chunk lane
    uint64_t cst;
    uint32_t clen, r, q;
    uint32_t w[33];
};

template <int WAVES>
struct Sweep {
    const Crc4Perm &crc;
    uint32_t *V, *HD;
    const uint32_t *Z;
    uint64_t base, end, src_len;
    uint32_t lane, rpr, n;
    const bhg_handle *handles;
    bhg_desc *out;

    __device__ __forceinline__ void prep(SwRound &R, uint32_t round, const bhg_handle &h) const {
        const uint32_t i = round * rpr + lane;
        R.mine = lane < rpr && i < n;
        R.inb = false;
        R.st = BHG_ST_OK;
        if (R.mine) {
            if (h.length == 0) R.st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) R.st = BHG_ST_INCOMPLETE;
            else R.inb = true;
        }
        R.p = base + h.offset;
        R.L = R.inb ? h.length : 0u;
        R.m = R.inb ? (R.L + 127) >> 7 : 0u;
        uint32_t incl = R.m;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += t;
        }
        R.cs = incl - R.m;
        R.M = __shfl(incl, 63, 64);
        chunk(R, 0);
    }
    // map lane -> (record, chunk) for pass pb and issue its window loads
    __device__ __forceinline__ void chunk(SwRound &R, uint32_t pb) const {
        const uint32_t c = pb + lane;
        uint32_t r = 0;
        for (uint32_t j = 1; j < rpr; j++) r += (uint32_t)__shfl(R.cs, j, 64) <= c ? 1u : 0u;
        const uint64_t pr = shfl64(R.p, r);
        const uint32_t Lr = __shfl(R.L, r, 64), mr = __shfl(R.m, r, 64), csr = __shfl(R.cs, r, 64);
        const uint32_t q = c - csr;
        const uint32_t hs = Lr - 128u * (mr - 1);
        R.r = r;
        R.q = q;
        R.cst = pr + (q ? hs + 128u * (q - 1) : 0u);
        R.clen = c < R.M ? (q ? 128u : hs) : 0u;
        if (R.clen) {
            const uint64_t a0 = R.cst & ~3ull;
            if (a0 + 132 <= end) {
#pragma unroll
                for (uint32_t qq = 0; qq < 8; qq++) {
                    const u32x4 x = gld<u32x4_a4>(a0 + 16 * qq);
                    R.w[4 * qq] = x.x; R.w[4 * qq + 1] = x.y; R.w[4 * qq + 2] = x.z; R.w[4 * qq + 3] = x.w;
                }
                R.w[32] = gld<uint32_t>(a0 + 128);
            } else {
#pragma unroll
                for (uint32_t t = 0; t <= 32; t++) R.w[t] = ld32_safe(a0 + 4 * t, end);
            }
        }
    }
    __device__ __forceinline__ void finish(SwRound &R, uint32_t round) const {
        uint32_t S = 0;
        for (uint32_t pb = 0;;) {
            uint32_t v = R.q == 0 ? 0xffffffffu : 0u;
            const uint32_t sh = (uint32_t)(R.cst & 3);
            if (R.clen) {
                const uint32_t nw = R.clen >> 2, tail = R.clen & 3;
#pragma unroll
                for (uint32_t t = 0; t < 32; t++)
                    if (t < nw) v = crc.word(v, __builtin_amdgcn_alignbyte(R.w[t + 1], R.w[t], sh));
                if (tail) v = crc.partial(v, ldu32(R.cst + 4 * nw, end), tail);
                if (R.q == 0 && pb == 0) {  // head chunk: export record bytes [0, 64)
#pragma unroll
                    for (uint32_t t = 0; t < 16; t++) HD[R.r * 16 + t] = __builtin_amdgcn_alignbyte(R.w[t + 1], R.w[t], sh);
                }
            }
            V[lane] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (R.m) {
                const uint32_t q0 = pb > R.cs ? pb - R.cs : 0u;
                const uint32_t q1 = min(R.m, pb + 64 - R.cs);
                for (uint32_t qq = q0; qq < q1 && R.cs + qq >= pb; qq++) {
                    const uint32_t x = V[R.cs + qq - pb];
                    S = (qq == 0 ? 0u : (Z[S & 255u] ^ Z[256 + ((S >> 8) & 255u)] ^ Z[512 + ((S >> 16) & 255u)] ^ Z[768 + (S >> 24)])) ^ x;
                }
            }
            pb += 64;
            if (pb >= R.M) break;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            chunk(R, pb);  // long rounds: further passes load synchronously
        }
        if (R.mine) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, R.st};
            if (R.inb) {
                const uint32_t L = R.L;
                uint32_t rw[15];
#pragma unroll
                for (int j = 0; j < 15; j++) rw[j] = HD[lane * 16 + j];
                RecHead H;
                if (L < 64) {
                    H.parse(R.p, L, end);
                } else {
                    // same as RecHead::parse over the exported words
                    H.k = rw[0];
                    H.v = rw[1];
                    H.fn = rw[2];
                    H.valid = H.k != 0 && H.v != 0 && (uint64_t)12 + H.k + H.v == (uint64_t)L;
                    H.key_len = 0;
                    H.fnv = BHG_FNV_OFFSET;
                    H.trailer = 255;
                    if (H.valid && H.k >= 8) {
                        H.key_len = H.k - 8;
                        if (H.key_len <= 36) {
                            PrefixL P;
#pragma unroll
                            for (int j = 0; j < 15; j++) P.rw[j] = rw[j];
                            H.fnv = P.fnv_key(H.key_len);
                            H.trailer = (uint64_t)P.word_at(12 + H.key_len) | ((uint64_t)P.word_at(16 + H.key_len) << 32);
                        } else {
                            H.fnv = fnv1_range(R.p + 12, H.key_len, end);
                            H.trailer = ldu64(R.p + 12 + H.k - 8, end);
                        }
                    }
                }
                d = H.desc(crc_mask(~S));
            }
            store_descL(out + round * rpr + lane, d);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
};

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_sweep2(const uint8_t *__restrict__ src, uint64_t src_len,
                                                       const bhg_handle *__restrict__ handles, uint32_t n,
                                                       bhg_desc *__restrict__ out, const uint32_t *__restrict__ gtab,
                                                       uint32_t rpr) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[1024];
    __shared__ uint32_t V[WAVES][64];
    __shared__ uint32_t HD[WAVES][16 * 16];
    Crc4Perm::fill(T, gtab);
    for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) Z[t] = gtab[1024 + t];
    __syncthreads();
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Sweep<WAVES> S{crc, V[wave], HD[wave], Z, (uint64_t)src, (uint64_t)src + src_len, src_len, lane, rpr, n, handles, out};
    const uint32_t nrounds = (n + rpr - 1) / rpr;
    const uint32_t W = gridDim.x * WAVES;
    auto hload = [&](uint32_t rd) {
        bhg_handle h = {0, 0, 0};
        if (rd < nrounds && lane < rpr && rd * rpr + lane < n) h = handles[rd * rpr + lane];
        return h;
    };
    uint32_t round = blockIdx.x * WAVES + wave;
    if (round >= nrounds) return;
    bhg_handle h1 = hload(round + W);
    SwRound A, B;
    S.prep(A, round, hload(round));
    for (;;) {
        const uint32_t rB = round + W;
        const bhg_handle h2 = hload(rB + W);
        if (rB < nrounds) S.prep(B, rB, h1);
        S.finish(A, round);
        if (rB >= nrounds) break;
        const uint32_t rA = rB + W;
        h1 = hload(rA + W);
        if (rA < nrounds) S.prep(A, rA, h2);
        S.finish(B, rB);
        if (rA >= nrounds) break;
        round = rA;
    }
}


// ============================================================== E7: per-lane walk, head/tail first, tail CRC shifted
// Lane per record.  The head line (p & ~127) and tail line ((E-1) & ~127) are
// loaded first -- in the same instructions as the neighbouring lanes' tail /
// head, which are the same physical lines -- and absorbed at once: the head
// from 0xFFFFFFFF, the tail from 0 (crc_0(T)).  The interior lines, owned by
// this lane alone, are walked in between, and the record CRC is
// Z_|T|(state) ^ crc_0(T) (GF(2) linearity), with Z_|T| from 6 shift tables
// (4..128 B) and up to 3 byte steps.
struct ZShift {
    const uint32_t *ZS;  // 6 x 1024 words: Z_4, Z_8, ..., Z_128
    template <class Tab>
    __device__ __forceinline__ uint32_t apply(const Tab &T, uint32_t c, uint32_t nbytes) const {
        const uint32_t b = nbytes & 3u, a = nbytes >> 2;
#pragma unroll
        for (uint32_t s = 0; s < 3; s++) {
            const uint32_t x = T.step(c);
            c = s < b ? x : c;
        }
#pragma unroll
        for (uint32_t j = 0; j < 6; j++) {
            if ((a >> j) & 1u) {
                const uint32_t *Z = ZS + j * 1024;
                c = Z[c & 255u] ^ Z[256 + ((c >> 8) & 255u)] ^ Z[512 + ((c >> 16) & 255u)] ^ Z[768 + (c >> 24)];
            }
        }
        return c;
    }
};

template <int WG, int MODE>
__global__ __launch_bounds__(WG) void k_lane5(const uint8_t *__restrict__ src, uint64_t src_len,
                                              const bhg_handle *__restrict__ handles, uint32_t n,
                                              bhg_desc *__restrict__ out, const uint32_t *__restrict__ gtab) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t ZS[6 * 1024];
    Crc4Perm::fill(T, gtab);
    for (uint32_t t = threadIdx.x; t < 6 * 1024; t += blockDim.x) ZS[t] = gtab[1024 + t];
    __syncthreads();
    const Crc4Perm crc(T);
    const ZShift zs{ZS};
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bhg_handle hn = {0, 0, 0};
    if (i < n) hn = handles[i];
    for (; i < n; i += stride) {
        const bhg_handle h = hn;
        if (i + stride < n) hn = handles[i + stride];
        DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, BHG_ST_OK};
        if (h.length == 0) {
            d.status = BHG_ST_ILLEGAL_LENGTH;
        } else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) {
            d.status = BHG_ST_INCOMPLETE;
        } else {
            const uint64_t p = base + h.offset, e = p + h.length;
            const uint64_t ha = p & ~127ull, ta = (e - 1) & ~127ull;
            uint32_t c, t0 = 0;
            {
                u32x4 H[8];
                load_line(H, ha, base, end);
                if ((MODE & 3) == 1) {
                    c = 0;
#pragma unroll
                    for (int t = 0; t < 32; t++) c ^= lw(H, t);
                } else {
                    c = absorb_line(crc, 0xffffffffu, H, (uint32_t)(p - ha), ta == ha ? (uint32_t)(e - ha) : 128u);
                }
            }
            if (ta != ha) {
                u32x4 Tl[8];
                load_line(Tl, ta, base, end);
                if ((MODE & 3) == 1) {
#pragma unroll
                    for (int t = 0; t < 32; t++) t0 ^= lw(Tl, t);
                } else {
                    t0 = absorb_line(crc, 0u, Tl, 0u, (uint32_t)(e - ta));
                }
            }
            RecHead R;
            R.valid = false;
            if (!(MODE & 4)) R.parse(p, h.length, end);
            if (ta != ha) {
                u32x4 A[8], B[8];
                uint64_t w = ha + 128;
                if (w < ta) load_line(A, w, base, end);
                while (w < ta) {
                    const uint64_t w1 = w + 128;
                    if (w1 < ta) load_line(B, w1, base, end);
                    if ((MODE & 3) == 1) {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = ((c << 1) | (c >> 31)) ^ lw(A, t);
                    } else {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = crc.word(c, lw(A, t));
                    }
                    if (w1 >= ta) break;
                    const uint64_t w2 = w1 + 128;
                    if (w2 < ta) load_line(A, w2, base, end);
                    if ((MODE & 3) == 1) {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = ((c << 1) | (c >> 31)) ^ lw(B, t);
                    } else {
#pragma unroll
                        for (int t = 0; t < 32; t++) c = crc.word(c, lw(B, t));
                    }
                    w = w2;
                }
                c = ((MODE & 3) == 1 ? c : zs.apply(crc, c, (uint32_t)(e - ta))) ^ t0;
            }
            d = R.desc(crc_mask(~c));
        }
        if (MODE & 8) reinterpret_cast<uint32_t *>(out + i)[8] = d.crc;
        else store_descL(out + i, d);
    }
}

// ============================================================== E2: chunked wave-cooperative CRC
// A wave owns a tile of 64 handles.  Every record is cut into CH-byte chunks
// aligned to its END (chunk 0 = the head, 1..CH bytes); the tile's chunks are
// dealt to the lanes 64 at a time in stream order, so one round of a wave
// reads one contiguous run of bytes.  Each lane CRCs its chunk from zero
// state (the head chunk from 0xFFFFFFFF), shifts it by CH*j zero bytes (j =
// chunks after it; binary decomposition over NB shift tables) and xors it
// into the record's LDS accumulator.
template <int CH, int NB, int WAVES, int MODE>
__global__ __launch_bounds__(64 * WAVES) void k_chunk(const uint8_t *__restrict__ src, uint64_t src_len,
                                                      const bhg_handle *__restrict__ handles, uint32_t n,
                                                      bhg_desc *__restrict__ out, const uint32_t *__restrict__ gshift) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t S[NB * 1024];
    __shared__ uint32_t CS[WAVES][66];
    __shared__ uint32_t ACC[WAVES][64];
    Crc4Perm::fill(T);
    for (uint32_t t = threadIdx.x; t < NB * 1024; t += blockDim.x) S[t] = gshift[t];
    __syncthreads();
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    constexpr uint32_t LMAX = (uint32_t)CH << NB;
    constexpr uint32_t NQ = CH / 16;
    for (uint32_t tile = blockIdx.x * WAVES + wave; tile < ntiles; tile += gridDim.x * WAVES) {
        const uint32_t i = tile * 64 + lane;
        bhg_handle h = {0, 0, 0};
        if (i < n) h = handles[i];
        bool inb = false;
        uint32_t st = BHG_ST_OK;
        if (i < n) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint64_t p = base + h.offset;
        const uint32_t L = inb ? h.length : 0u;
        RecHead H;
        H.valid = false;
        if (inb && !(MODE & 4)) H.parse(p, L, end);
        const uint32_t m = (inb && L <= LMAX) ? (L + CH - 1) / CH : 0u;
        uint32_t incl = m;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += t;
        }
        const uint32_t M = __shfl(incl, 63, 64);
        CS[wave][lane] = incl - m;
        if (lane == 63) CS[wave][64] = incl;
        ACC[wave][lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t r0 = 0; r0 < M; r0 += 64) {
            const uint32_t ci = r0 + lane;
            const bool act = ci < M;
            uint32_t r = 0;
#pragma unroll
            for (uint32_t s = 32; s > 0; s >>= 1)
                if (CS[wave][r + s] <= ci) r += s;
            const uint32_t csr = CS[wave][r];
            const uint64_t pr = shfl64(p, r);
            const uint32_t Lr = __shfl(L, r, 64), mr = __shfl(m, r, 64);
            const uint32_t q = ci - csr;
            const uint32_t hs = Lr - CH * (mr - 1);
            const uint32_t j = mr - 1 - q;
            const uint64_t cst = pr + (q ? hs + CH * (q - 1) : 0u);
            const uint32_t clen = act ? (q ? (uint32_t)CH : hs) : 0u;
            uint32_t c = (q == 0) ? 0xffffffffu : 0u;
            if ((MODE & 3) == 2) {  // compute only: synthetic words
#pragma unroll
                for (uint32_t t = 0; t < CH / 4; t++)
                    if (4 * t < clen) c = crc.word(c, (uint32_t)cst + t * 0x9e3779b9u);
            } else if (clen) {
                const uint64_t a0 = cst & ~3ull;
                const uint32_t sh = (uint32_t)(cst & 3);
                uint32_t w[CH / 4 + 1];
                if (a0 + CH + 4 <= end) {
#pragma unroll
                    for (uint32_t qq = 0; qq < NQ; qq++) {
                        const u32x4 v = gld<u32x4_a4>(a0 + 16 * qq);
                        w[4 * qq] = v.x; w[4 * qq + 1] = v.y; w[4 * qq + 2] = v.z; w[4 * qq + 3] = v.w;
                    }
                    w[CH / 4] = gld<uint32_t>(a0 + CH);
                } else {
#pragma unroll
                    for (uint32_t t = 0; t <= CH / 4; t++) w[t] = ld32_safe(a0 + 4 * t, end);
                }
                const uint32_t nw = clen >> 2, tail = clen & 3;
                if ((MODE & 3) == 1) {
#pragma unroll
                    for (uint32_t t = 0; t < CH / 4; t++)
                        if (t < nw) c = ((c << 1) | (c >> 31)) ^ __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                } else {
#pragma unroll
                    for (uint32_t t = 0; t < CH / 4; t++)
                        if (t < nw) c = crc.word(c, __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh));
                }
                if (tail) {
                    const uint64_t tp = cst + 4 * nw;
                    c = crc.partial(c, ldu32(tp, end), tail);
                }
            }
            if ((MODE & 3) != 1) {
#pragma unroll
                for (uint32_t b = 0; b < NB; b++) {
                    if ((j >> b) & 1u) {
                        const uint32_t *Sb = S + b * 1024;
                        c = Sb[c & 255u] ^ Sb[256 + ((c >> 8) & 255u)] ^ Sb[512 + ((c >> 16) & 255u)] ^ Sb[768 + (c >> 24)];
                    }
                }
            }
            if (act) atomicXor(&ACC[wave][r], c);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (i < n) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) {
                uint32_t state = ACC[wave][lane];
                if (L > LMAX) state = crc_range_a<8, Crc4Perm, true>(crc, 0xffffffffu, p, L, end);
                d = H.desc(crc_mask(~state));
            }
            if (MODE & 8) reinterpret_cast<uint32_t *>(out + i)[8] = d.crc;
            else store_descL(out + i, d);
        }
    }
}


// ============================================================== E3: braided (dword-interleaved) CRC
// G lanes per record, 64/G records per group step.  The record is viewed as
// D dwords after z = (-L) & 3 leading zero pad bytes (free for a zero-init
// CRC); chain g (lane g of the group) takes the dwords whose index from the
// END is = g (mod G), so step k of the group reads G consecutive dwords of
// each record (coalesced).  Each dword is absorbed with braid tables that
// fold the G-1 dwords of the other chains (Z_{4(G-1)}), so chain g's residue
// is "as of" L' + 4(G-1-g); a log2(G)-level tree with fixed backward shifts
// Z_{-4*2^s} brings all chains to the record end.  The init 0xFFFFFFFF is
// xored into record bytes [0, 4).
template <int G, int WAVES, int U, int MODE>
__global__ __launch_bounds__(64 * WAVES) void k_braid(const uint8_t *__restrict__ src, uint64_t src_len,
                                                      const bhg_handle *__restrict__ handles, uint32_t n,
                                                      bhg_desc *__restrict__ out, const uint32_t *__restrict__ gtab) {
    constexpr int LG = G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3 : G == 16 ? 4 : 5;
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t S[LG * 1024];
    __shared__ uint32_t RES[WAVES][64];
    Crc4Perm::fill(T, gtab);
    for (uint32_t t = threadIdx.x; t < LG * 1024; t += blockDim.x) S[t] = gtab[1024 + t];
    __syncthreads();
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t g = lane % G, rr = lane / G;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    for (uint32_t tile = blockIdx.x * WAVES + wave; tile < ntiles; tile += gridDim.x * WAVES) {
        const uint32_t i = tile * 64 + lane;
        bhg_handle h = {0, 0, 0};
        if (i < n) h = handles[i];
        bool inb = false;
        uint32_t st = BHG_ST_OK;
        if (i < n) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint64_t p = base + h.offset;
        const uint32_t L = inb ? h.length : 0u;
        RecHead H;
        if (inb) H.parse(p, L, end);
        // braid-eligible: L >= 4 and the padded start p - z stays inside src
        const uint32_t zz = (0u - L) & 3u;
        const bool br = inb && L >= 4 && h.offset >= zz;
        const uint32_t Dm = br ? (L + zz) >> 2 : 0u;
        const uint64_t e4 = p + L;  // record end; dword d (from the end) at e4 - 4(d+1)
#pragma unroll 1
        for (uint32_t grp = 0; grp < G; grp++) {
            const uint32_t r = grp * (64 / G) + rr;
            const uint64_t er = shfl64(e4, r);
            const uint32_t D = __shfl(Dm, r, 64), Lr = __shfl(L, r, 64);
            uint32_t Kmax = (D + G - 1) / G;
#pragma unroll
            for (int o = G; o < 64; o <<= 1) Kmax = max(Kmax, (uint32_t)__shfl_xor(Kmax, o, 64));
            const uint32_t K = D > g ? (D - 1 - g) / G + 1 : 0u;
            // chain g's k-th dword (k = 0..K-1, in stream order) has index-from-end g + G(K-1-k)
            uint32_t c = 0;
            for (uint32_t k0 = 0; k0 < Kmax; k0 += U) {
                uint32_t w[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t k = k0 + u;
                    w[u] = 0;
                    if (k < K) {
                        const uint32_t d = g + G * (K - 1 - k);
                        const uint64_t a = er - 4ull * (d + 1);
                        w[u] = gld<uint32_t>(a);
                    }
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t k = k0 + u;
                    if (k < K) {
                        const uint32_t d = g + G * (K - 1 - k);
                        uint32_t x = w[u];
                        // record bytes [0,4) carry the init; leading pad bytes are zero
                        const uint32_t zr = (0u - Lr) & 3u;
                        if (d == D - 1) x = (x & (0xffffffffu << (8 * zr))) ^ (0xffffffffu << (8 * zr));
                        if (zr && d == D - 2) x ^= 0xffffffffu >> (32 - 8 * zr);
                        if (MODE == 1) c = ((c << 1) | (c >> 31)) ^ x;
                        else c = crc.word(c, x);
                    }
                }
            }
            if (MODE != 1) {
#pragma unroll
                for (int s = 0; s < LG; s++) {
                    const uint32_t *Sb = S + s * 1024;
                    const uint32_t sh = Sb[c & 255u] ^ Sb[256 + ((c >> 8) & 255u)] ^ Sb[512 + ((c >> 16) & 255u)] ^ Sb[768 + (c >> 24)];
                    const uint32_t a = ((g >> s) & 1u) ? c : sh;
                    c = a ^ (uint32_t)__shfl_xor(a, 1 << s, 64);
                }
            } else {
#pragma unroll
                for (int s = 0; s < LG; s++) c ^= (uint32_t)__shfl_xor(c, 1 << s, 64);
            }
            if (g == 0) RES[wave][r] = c;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (i < n) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) {
                uint32_t state = RES[wave][lane];
                if (!br) state = crc_range_a<8, Crc4Perm, true>(crc, 0xffffffffu, p, L, end);  // needs plain table!
                d = H.desc(crc_mask(~state));
            }
            store_descL(out + i, d);
        }
    }
}


// ============================================================== E2b: chunked, software-pipelined
// Same math as k_chunk; the windows of round k+1 are loaded while round k is
// absorbed (two register buffers, explicit ping-pong).
template <int CH, int NB, int WAVES, int MODE>
__global__ __launch_bounds__(64 * WAVES) void k_chunk2(const uint8_t *__restrict__ src, uint64_t src_len,
                                                       const bhg_handle *__restrict__ handles, uint32_t n,
                                                       bhg_desc *__restrict__ out, const uint32_t *__restrict__ gshift) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t S[NB * 1024];
    __shared__ uint32_t CS[WAVES][66];
    __shared__ uint32_t ACC[WAVES][64];
    Crc4Perm::fill(T);
    for (uint32_t t = threadIdx.x; t < NB * 1024; t += blockDim.x) S[t] = gshift[t];
    __syncthreads();
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    constexpr uint32_t LMAX = (uint32_t)CH << NB;
    constexpr uint32_t NQ = CH / 16;
    constexpr uint32_t NW = CH / 4;
    struct Job {
        uint64_t cst;
        uint32_t clen, j, r, head;
    };
    for (uint32_t tile = blockIdx.x * WAVES + wave; tile < ntiles; tile += gridDim.x * WAVES) {
        const uint32_t i = tile * 64 + lane;
        bhg_handle h = {0, 0, 0};
        if (i < n) h = handles[i];
        bool inb = false;
        uint32_t st = BHG_ST_OK;
        if (i < n) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint64_t p = base + h.offset;
        const uint32_t L = inb ? h.length : 0u;
        const uint32_t m = (inb && L <= LMAX) ? (L + CH - 1) / CH : 0u;
        uint32_t incl = m;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += t;
        }
        const uint32_t M = __shfl(incl, 63, 64);
        CS[wave][lane] = incl - m;
        if (lane == 63) CS[wave][64] = incl;
        ACC[wave][lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        auto prep = [&](uint32_t r0) {
            Job J;
            const uint32_t ci = r0 + lane;
            uint32_t r = 0;
#pragma unroll
            for (uint32_t s2 = 32; s2 > 0; s2 >>= 1)
                if (CS[wave][r + s2] <= ci) r += s2;
            const uint32_t csr = CS[wave][r];
            const uint64_t pr = shfl64(p, r);
            const uint32_t Lr = __shfl(L, r, 64), mr = __shfl(m, r, 64);
            const uint32_t q = ci - csr;
            const uint32_t hs = Lr - CH * (mr - 1);
            J.j = mr - 1 - q;
            J.cst = pr + (q ? hs + CH * (q - 1) : 0u);
            J.clen = ci < M ? (q ? (uint32_t)CH : hs) : 0u;
            J.r = r;
            J.head = q == 0;
            return J;
        };
        auto issue = [&](const Job &J, uint32_t *w) {
            if (J.clen) {
                const uint64_t a0 = J.cst & ~3ull;
                if (a0 + CH + 4 <= end) {
#pragma unroll
                    for (uint32_t qq = 0; qq < NQ; qq++) {
                        const u32x4 v = gld<u32x4_a4>(a0 + 16 * qq);
                        w[4 * qq] = v.x; w[4 * qq + 1] = v.y; w[4 * qq + 2] = v.z; w[4 * qq + 3] = v.w;
                    }
                    w[NW] = gld<uint32_t>(a0 + CH);
                } else {
#pragma unroll
                    for (uint32_t t = 0; t <= NW; t++) w[t] = ld32_safe(a0 + 4 * t, end);
                }
            }
        };
        auto absorb = [&](const Job &J, const uint32_t *w) {
            uint32_t c = J.head ? 0xffffffffu : 0u;
            if (J.clen) {
                const uint32_t sh = (uint32_t)(J.cst & 3);
                const uint32_t nw = J.clen >> 2, tail = J.clen & 3;
                if (MODE == 1) {
#pragma unroll
                    for (uint32_t t = 0; t < NW; t++)
                        if (t < nw) c = ((c << 1) | (c >> 31)) ^ __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                } else {
#pragma unroll
                    for (uint32_t t = 0; t < NW; t++)
                        if (t < nw) c = crc.word(c, __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh));
                }
                if (tail) c = crc.partial(c, ldu32(J.cst + 4 * nw, end), tail);
                if (MODE != 1) {
#pragma unroll
                    for (uint32_t b = 0; b < NB; b++) {
                        if ((J.j >> b) & 1u) {
                            const uint32_t *Sb = S + b * 1024;
                            c = Sb[c & 255u] ^ Sb[256 + ((c >> 8) & 255u)] ^ Sb[512 + ((c >> 16) & 255u)] ^ Sb[768 + (c >> 24)];
                        }
                    }
                }
                atomicXor(&ACC[wave][J.r], c);
            }
        };
        uint32_t WA[NW + 1], WB[NW + 1];
        Job JA = prep(0), JB;
        if (M) issue(JA, WA);
        for (uint32_t r0 = 0; r0 < M; r0 += 128) {
            const bool moreB = r0 + 64 < M;
            if (moreB) { JB = prep(r0 + 64); issue(JB, WB); }
            absorb(JA, WA);
            if (!moreB) break;
            const bool moreA = r0 + 128 < M;
            if (moreA) { JA = prep(r0 + 128); issue(JA, WA); }
            absorb(JB, WB);
        }
        RecHead H;
        if (inb) H.parse(p, L, end);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (i < n) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) {
                uint32_t state = ACC[wave][lane];
                if (L > LMAX) state = crc_range_a<8, Crc4Perm, true>(crc, 0xffffffffu, p, L, end);
                d = H.desc(crc_mask(~state));
            }
            store_descL(out + i, d);
        }
    }
}

// ============================================================== diag: linear stream read
template <int UNR>
__global__ __launch_bounds__(256) void k_stream(const uint8_t *__restrict__ src, uint64_t src_len,
                                                bhg_desc *__restrict__ out) {
    const uint64_t base = (uint64_t)src;
    const uint64_t nvec = src_len / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride * UNR) {
        u32x4 x[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++)
            x[u] = v + u * stride < nvec ? gld<u32x4>(base + 16 * (v + u * stride)) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < UNR; u++) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    }
    if (acc == 0x12345678u) reinterpret_cast<uint32_t *>(out)[threadIdx.x] = acc;
}


// diag: wave-contiguous tiles of TB bytes, coalesced 1 KiB instructions; wave w
// takes tiles w, w + W, ... (concurrent span = W * TB)
template <int TB>
__global__ __launch_bounds__(256) void k_tiles(const uint8_t *__restrict__ src, uint64_t src_len, bhg_desc *__restrict__ out) {
    const uint64_t base = (uint64_t)src;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4, w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t ntiles = src_len / TB;
    uint32_t acc = 0;
    for (uint64_t t = w0; t < ntiles; t += W) {
        const uint64_t a = base + t * TB + 16 * lane;
#pragma unroll 4
        for (uint32_t o = 0; o < TB; o += 1024) {
            const u32x4 x = gld<u32x4>(a + o);
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
        }
    }
    if (acc == 0x12345678u) reinterpret_cast<uint32_t *>(out)[threadIdx.x] = acc;
}
// diag: per-lane contiguous regions of RB bytes (16 B per lane per
// instruction, 64 distinct regions per instruction); lane-regions ordered
// lane-major within a wave tile of 64 * RB bytes
template <int RB>
__global__ __launch_bounds__(256) void k_lanes(const uint8_t *__restrict__ src, uint64_t src_len, bhg_desc *__restrict__ out) {
    const uint64_t base = (uint64_t)src;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4, w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t ntiles = src_len / (64ull * RB);
    uint32_t acc = 0;
    for (uint64_t t = w0; t < ntiles; t += W) {
        const uint64_t a = base + t * 64ull * RB + (uint64_t)lane * RB;
#pragma unroll 8
        for (uint32_t o = 0; o < RB; o += 16) {
            const u32x4 x = gld<u32x4>(a + o);
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
        }
    }
    if (acc == 0x12345678u) reinterpret_cast<uint32_t *>(out)[threadIdx.x] = acc;
}


// diag: per-lane record walk: lane reads RL bytes starting at OFF + lane_rec * RL
// using 16 B loads at (4-aligned) addresses, MODE 0: from p & ~3 (unaligned
// dwordx4), MODE 1: from 16-aligned windows covering [p, p + RL)
template <int RL, int MODE>
__global__ __launch_bounds__(256) void k_lrec(const uint8_t *__restrict__ src, uint64_t src_len, bhg_desc *__restrict__ out) {
    const uint64_t base = (uint64_t)src;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4, w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t ntiles = src_len / (64ull * RL) - 1;
    uint32_t acc = 0;
    for (uint64_t t = w0; t < ntiles; t += W) {
        const uint64_t p = base + (t * 64ull + lane) * RL;
        const uint64_t a = MODE == 0 ? (p & ~3ull) : MODE == 1 ? (p & ~15ull) : (p & ~127ull);
        const uint64_t e = p + RL;
#pragma unroll 8
        for (uint64_t o = a; o < e; o += 16) {
            const u32x4 x = gld<u32x4_a4>(o);
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
        }
    }
    if (acc == 0x12345678u) reinterpret_cast<uint32_t *>(out)[threadIdx.x] = acc;
}


// diag: chunk pattern, lane l reads CH bytes at T + CH*l + OFF; MODE 0: dwordx4 from
// (addr & ~3), MODE 1: dwordx4 from (addr & ~15)
template <int CH, int OFF, int MODE>
__global__ __launch_bounds__(256) void k_cdiag(const uint8_t *__restrict__ src, uint64_t src_len, bhg_desc *__restrict__ out) {
    const uint64_t base = (uint64_t)src;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4, w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t ntiles = src_len / (64ull * CH) - 1;
    uint32_t acc = 0;
    for (uint64_t t = w0; t < ntiles; t += W) {
        const uint64_t p = base + (t * 64ull + lane) * CH + OFF;
        const uint64_t a = MODE == 0 ? (p & ~3ull) : (p & ~15ull);
        u32x4 x[CH / 16 + 1];
#pragma unroll
        for (int q = 0; q <= CH / 16; q++) x[q] = gld<u32x4_a4>(a + 16 * q);
#pragma unroll
        for (int q = 0; q <= CH / 16; q++) acc ^= x[q].x ^ x[q].y ^ x[q].z ^ x[q].w;
    }
    if (acc == 0x12345678u) reinterpret_cast<uint32_t *>(out)[threadIdx.x] = acc;
}


// diag: line-grid rounds over each 64-handle tile's byte range (loads + xor only)
template <int WAVES, int PF, int TR = 64>
__global__ __launch_bounds__(64 * WAVES) void k_gridload(const uint8_t *__restrict__ src, uint64_t src_len,
                                                         const bhg_handle *__restrict__ handles, uint32_t n,
                                                         bhg_desc *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)src;
    const uint32_t ntiles = (n + TR - 1) / TR;
    for (uint32_t tile = blockIdx.x * WAVES + wave; tile < ntiles; tile += gridDim.x * WAVES) {
        const uint32_t i = tile * TR + lane;
        bhg_handle h = {0, 0, 0};
        if (i < n && lane < TR) h = handles[i];
        const uint64_t p = base + h.offset, e = p + h.length;
        const uint32_t last = min((uint32_t)TR - 1, n - 1 - tile * TR);
        const uint64_t a0 = shfl64(p, 0) & ~127ull, ee = shfl64(e, last);
        const uint32_t nl = (uint32_t)((ee - a0 + 127) >> 7);
        uint32_t acc = 0;
        u32x4 A[8], B[8];
        auto ld = [&](u32x4 *v, uint32_t c) {
            if (c < nl) {
#pragma unroll
                for (int q = 0; q < 8; q++) v[q] = gld<u32x4>(a0 + 128ull * c + 16 * q);
            } else {
#pragma unroll
                for (int q = 0; q < 8; q++) v[q] = u32x4{0, 0, 0, 0};
            }
        };
        auto fold = [&](const u32x4 *v) {
#pragma unroll
            for (int q = 0; q < 8; q++) acc = ((acc << 1) | (acc >> 31)) ^ v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
        };
        if (PF) {
            ld(A, lane);
            for (uint32_t c0 = 0; c0 < nl; c0 += 128) {
                ld(B, c0 + 64 + lane);
                fold(A);
                if (c0 + 64 >= nl) break;
                ld(A, c0 + 128 + lane);
                fold(B);
            }
        } else {
            for (uint32_t c0 = 0; c0 < nl; c0 += 64) {
                ld(A, c0 + lane);
                fold(A);
            }
        }
        if (i < n && lane < TR) reinterpret_cast<uint32_t *>(out + i)[8] = acc;
    }
}


// diag: pure CRC compute, NCH independent chains per lane, NW words per chain
// (data synthesised in registers), total work = the batch's words
template <int NCH, int TBL>
__global__ __launch_bounds__(1024) void k_ccompute(const uint8_t *__restrict__ src, uint64_t src_len, bhg_desc *__restrict__ out,
                                                  const uint32_t *__restrict__ gtab) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    Crc4Perm::fill(T, gtab);
    __syncthreads();
    const Crc4Perm crc(T);
    const uint64_t words = src_len / 4;
    const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t per = words / lanes / NCH;   // words per chain
    uint32_t c[NCH];
#pragma unroll
    for (int k = 0; k < NCH; k++) c[k] = threadIdx.x * 7 + k;
    uint32_t w = blockIdx.x * 0x9e3779b9u + threadIdx.x;
    for (uint64_t t = 0; t < per; t++) {
        w = w * 1664525u + 1013904223u;
#pragma unroll
        for (int k = 0; k < NCH; k++) c[k] = crc.word(c[k], w + k);
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < NCH; k++) x ^= c[k];
    if (x == 0x12345678u) reinterpret_cast<uint32_t *>(out)[threadIdx.x] = x;
}



// header / key / trailer / FNV-1 from a record staged in LDS at byte offset a
// (key_len <= 36 from 13 LDS dwords; longer keys fall back to global reads)
__device__ __forceinline__ uint32_t keep_from(int32_t x) {  // bytes b >= x of a dword (x clamped to [0, 4])
    const int32_t c = x < 0 ? 0 : (x > 4 ? 4 : x);
    return (uint32_t)(0xffffffffull << (8 * c));
}
__device__ __forceinline__ uint32_t lds_u32(const uint8_t *B, uint32_t a) {
    const uint32_t *W = reinterpret_cast<const uint32_t *>(B + (a & ~3u));
    const uint32_t sh = a & 3u;
    return sh ? __builtin_amdgcn_alignbyte(W[1], W[0], sh) : W[0];
}
__device__ __forceinline__ void parse_lds(RecHead &H, const uint8_t *B, uint32_t a, uint64_t p, uint32_t L,
                                          uint64_t end) {
    H.k = lds_u32(B, a);
    H.v = lds_u32(B, a + 4);
    H.fn = lds_u32(B, a + 8);
    H.valid = L >= 12 && H.k != 0 && H.v != 0 && (uint64_t)12 + H.k + H.v == (uint64_t)L;
    H.key_len = 0;
    H.fnv = BHG_FNV_OFFSET;
    H.trailer = 255;
    if (H.valid && H.k >= 8) {
        H.key_len = H.k - 8;
        if (H.key_len <= 36) {
            uint32_t rw[11];
#pragma unroll
            for (uint32_t t = 0; t < 11; t++) rw[t] = lds_u32(B, a + 12 + 4 * t);
            uint32_t h = BHG_FNV_OFFSET;
#pragma unroll
            for (uint32_t t = 0; t < 9; t++)
#pragma unroll
                for (uint32_t b = 0; b < 4; b++) {
                    const uint32_t hn = (h * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * b)) & 0xffu);
                    h = 4 * t + b < H.key_len ? hn : h;
                }
            H.fnv = h;
            H.trailer = (uint64_t)lds_u32(B, a + 12 + H.key_len) | ((uint64_t)lds_u32(B, a + 16 + H.key_len) << 32);
        } else {
            H.fnv = fnv1_range(p + 12, H.key_len, end);
            H.trailer = ldu64(p + 12 + H.k - 8, end);
        }
    }
}

// ============================================================== E8: LDS-staged groups, striped chunk CRC
// A workgroup of G*S threads takes groups of G consecutive handles.  The
// group's byte span [lo16, hi) is loaded with coalesced dwordx4 loads (one
// group ahead, register staged) into an LDS buffer; every record is cut into
// CH-byte windows aligned to its END (window 0 holds the head, left-padded
// with zeros, and absorbs the 0xFFFFFFFF init by xoring it into the record's
// first 4 bytes).  Thread (r, j) = (t % G, t / G) takes windows q = m-1-j,
// m-1-j-S, ... of record r: each window's CRC (from 0) runs as 4 interleaved
// 32 B chains folded with Z_32; windows are Horner-folded with Z_{S*CH}, and
// the stripe's sum is moved to the record end with Z_{CH*j}.  The S stripe
// sums are xor-reduced through LDS; thread (r, 0) parses the header from LDS
// and writes the descriptor.  Lanes 0..31 of a 32-lane ds_read_b32 group are
// 32 different records: data reads are bank-conflict free at odd word strides.
// Groups whose span exceeds SPAN (scattered handles) fall back to a per-record
// global walk by thread (r, 0).
template <int G, int S, int CH, int R, int SPAN, int MODE>
__global__ __launch_bounds__(G * S) void k_stage(const uint8_t *__restrict__ src, uint64_t src_len,
                                                 const bhg_handle *__restrict__ handles, uint32_t n,
                                                 bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    static_assert(G == 32 && CH == 128 && (S & (S - 1)) == 0, "layout");
    constexpr uint32_t NT = G * S;
    constexpr uint32_t PAD = CH;                       // window 0 may start up to CH-1 bytes before the record
    constexpr uint32_t BUFB = PAD + SPAN + 16;
    constexpr uint32_t NV = (SPAN + 16 * NT - 1) / (16 * NT);  // dwordx4 per thread per group
    constexpr int SB = S == 8 ? 3 : S == 4 ? 2 : S == 2 ? 1 : 0;
    __shared__ __attribute__((aligned(16))) uint8_t ST[2][BUFB];
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Lds<R>::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[(2 + SB) * 1024];  // Z32, Z_{S*CH}, Z_{CH<<b}
    __shared__ uint32_t RED[S][G];
    __shared__ uint32_t MREL[2][G], ML[2][G], MFL[2][G];
    __shared__ uint64_t SPLO[2];
    __shared__ uint32_t SPNV[2];
    Crc4Lds<R>::fill(T);
    for (uint32_t t = threadIdx.x; t < (2 + SB) * 1024; t += NT) Z[t] = gz[t];
    const Crc4Lds<R> crc(T);
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t r = tid % G, j = tid / G;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ngroups = (n + G - 1) / G;
    const bool w0 = tid < 64;
    auto zapply = [&](const uint32_t *Zt, uint32_t c) {
        return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
    };
    // wave 0, lanes < G: handle of group g -> meta slot b (+ span)
    auto load_h = [&](uint32_t g) {
        bhg_handle h = {0, 0, 0};
        const uint32_t i = g * G + lane;
        if (w0 && lane < G && g < ngroups && i < n) h = handles[i];
        return h;
    };
    auto set_meta = [&](uint32_t g, const bhg_handle &h, int b) {
        if (!w0) return;
        const uint32_t i = g * G + lane;
        uint32_t fl = 0;  // bit0 valid index, bit1 inb, bit2 staged, bits 8.. status
        uint64_t lo = ~0ull, hi = 0;
        if (lane < G && g < ngroups && i < n) {
            fl = 1;
            if (h.length == 0) fl |= BHG_ST_ILLEGAL_LENGTH << 8;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) fl |= BHG_ST_INCOMPLETE << 8;
            else { fl |= 2; lo = h.offset; hi = h.offset + h.length; }
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t lo2 = shfl64(lo, lane ^ o), hi2 = shfl64(hi, lane ^ o);
            lo = lo2 < lo ? lo2 : lo;
            hi = hi2 > hi ? hi2 : hi;
        }
        const uint64_t lo16 = lo & ~15ull;
        const bool fits = hi > lo && hi - lo16 <= SPAN;
        if (lane < G) {
            MREL[b][lane] = (uint32_t)(h.offset - lo16);
            ML[b][lane] = h.length;
            MFL[b][lane] = fl | ((fits && (fl & 2) && h.length >= 4) ? 4u : 0u);
        }
        if (lane == 0) {
            SPLO[b] = lo16;
            SPNV[b] = fits ? (uint32_t)((hi - lo16 + 15) >> 4) : 0u;
        }
    };
    u32x4 pre[NV];
    auto issue = [&](int b) {
        const uint64_t a0 = base + SPLO[b];
        const uint32_t nv = SPNV[b];
        if (a0 + 16ull * nv <= end) {
#pragma unroll
            for (uint32_t k = 0; k < NV; k++) {
                const uint32_t v = tid + k * NT;
                if (v < nv) pre[k] = gld<u32x4>(a0 + 16ull * v);
            }
        } else {
            for (uint32_t k = 0; k < NV; k++) {
                const uint32_t v = tid + k * NT;
                const uint64_t a = a0 + 16ull * v;
                if (v < nv)
                    pre[k] = u32x4{ld32_safe(a, end), ld32_safe(a + 4, end), ld32_safe(a + 8, end), ld32_safe(a + 12, end)};
            }
        }
    };
    auto commit = [&](int b) {
        const uint32_t nv = SPNV[b];
#pragma unroll
        for (uint32_t k = 0; k < NV; k++) {
            const uint32_t v = tid + k * NT;
            if (v < nv) *reinterpret_cast<u32x4 *>(&ST[b][PAD + 16 * v]) = pre[k];
        }
    };
    uint32_t g = blockIdx.x;
    const uint32_t gs = gridDim.x;
    bhg_handle hn = load_h(g);
    set_meta(g, hn, 0);
    hn = load_h(g + gs);
    __syncthreads();
    issue(0);
    commit(0);
    set_meta(g + gs, hn, 1);
    hn = load_h(g + 2 * gs);
    __syncthreads();
    for (int cur = 0; g < ngroups; g += gs, cur ^= 1) {
        const int nxt = cur ^ 1;
        if (g + gs < ngroups) issue(nxt);
        // ---- striped window CRC over ST[cur]
        const uint32_t fl = MFL[cur][r];
        uint32_t acc = 0;
        if (fl & 4) {
            const uint32_t L = ML[cur][r], rel = MREL[cur][r];
            const uint32_t m = (L + CH - 1) / CH;
            if (j < m) {
                const uint32_t qmax = m - 1 - j;
                const uint32_t recend = PAD + rel + L;
                const uint32_t zlead = CH * m - L;  // zero bytes before the record in window 0
                for (int32_t q = (int32_t)(qmax % S); q <= (int32_t)qmax; q += S) {
                    const uint32_t A = recend - CH * (m - (uint32_t)q);
                    const uint32_t a0 = A & ~3u, sh = A & 3u;
                    const uint32_t *W = reinterpret_cast<const uint32_t *>(&ST[cur][a0]);
                    const int32_t zl = q == 0 ? (int32_t)zlead : -64;
                    uint32_t Wd[CH / 4 + 1];
#pragma unroll
                    for (uint32_t t = 0; t <= CH / 4; t++) Wd[t] = W[t];
                    uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
                    for (uint32_t t = 0; t < 8; t++) {
#pragma unroll
                        for (uint32_t k = 0; k < 4; k++) {
                            const uint32_t wi = 8 * k + t;
                            uint32_t w = __builtin_amdgcn_alignbyte(Wd[wi + 1], Wd[wi], sh);
                            const int32_t zz = zl - 4 * (int32_t)wi;  // record start relative to this word
                            const uint32_t k0 = keep_from(zz), k4 = keep_from(zz + 4);
                            w = (w & k0) ^ (k0 & ~k4);
                            c[k] = crc.word(c[k], w);
                        }
                    }
                    uint32_t v = zapply(Z, c[0]) ^ c[1];
                    v = zapply(Z, v) ^ c[2];
                    v = zapply(Z, v) ^ c[3];
                    acc = zapply(Z + 1024, acc) ^ v;
                }
#pragma unroll
                for (int b = 0; b < SB; b++)
                    if ((j >> b) & 1u) acc = zapply(Z + 2048 + 1024 * b, acc);
            }
        }
        RED[j][r] = acc;
        __syncthreads();
        if (j == 0 && (fl & 1)) {
            const uint32_t i = g * G + r;
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, fl >> 8};
            if (fl & 2) {
                const uint32_t L = ML[cur][r];
                const uint64_t p = base + SPLO[cur] + MREL[cur][r];
                uint32_t state;
                if (fl & 4) {
                    state = 0;
#pragma unroll
                    for (int s2 = 0; s2 < S; s2++) state ^= RED[s2][r];
                } else if (!(MODE & 1)) {
                    state = crc_range_a<8, Crc4Lds<R>, true>(crc, 0xffffffffu, p, L, end);
                } else {
                    state = 0;
                }
                RecHead H;
                if ((fl & 4) || (MODE & 1)) parse_lds(H, ST[cur], PAD + MREL[cur][r], p, L, end);
                else H.parse(p, L, end);
                d = H.desc(crc_mask(~state));
            }
            store_descL(out + i, d);
        }
        if (g + gs < ngroups) commit(nxt);
        set_meta(g + 2 * gs, hn, cur);
        hn = load_h(g + 3 * gs);
        __syncthreads();
    }
}


// ============================================================== E9: window-per-lane in registers, 8 lanes per record
// A wave takes groups of 8 consecutive handles; lane (r, j) = (lane / 8,
// lane % 8).  Record r is cut into its head [0, hl) (hl = L - 128 (m-1),
// 1..128 B) and m-1 full 128-B windows aligned to its end.  Lane j owns the
// windows q = m-1-j, m-1-j-8, ... (>= 1) and, when j == (m-1) % 8, the head.
// Each lane loads its windows straight into registers (132 B from a
// 4-aligned address: 64 lanes read one contiguous ~8.6 KB run per group),
// CRCs them (the head from 0xFFFFFFFF, full windows from 0), Horner-folds
// them with Z_1024, moves the sum to the record end with Z_{128 j} (three
// conditional table steps) and the 8 lanes xor-reduce.  The head lane parses
// the header / key / trailer / FNV-1 from its registers and writes the
// descriptor.  The next group's handles are prefetched one group ahead.
template <int WPB, int R, int MODE>
__global__ __launch_bounds__(64 * WPB) void k_win(const uint8_t *__restrict__ src, uint64_t src_len,
                                                  const bhg_handle *__restrict__ handles, uint32_t n,
                                                  bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Lds<R>::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[5 * 1024];  // Z1024, Z128, Z256, Z512, Z32
    Crc4Lds<R>::fill(T);
    for (uint32_t t = threadIdx.x; t < 5 * 1024; t += 64 * WPB) Z[t] = gz[t];
    const uint32_t *ZS32 = Z + 4096;
    __syncthreads();
    const Crc4Lds<R> crc(T);
    auto zapply = [&](const uint32_t *Zt, uint32_t c) {
        return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
    };
    const uint32_t lane = threadIdx.x & 63, r = lane >> 3, j = lane & 7;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ngroups = (n + 7) / 8;
    const uint32_t gstride = gridDim.x * WPB;
    uint32_t g = blockIdx.x * WPB + (threadIdx.x >> 6);
    bhg_handle hn = {0, 0, 0};
    if (g < ngroups && g * 8 + r < n) hn = handles[g * 8 + r];
    for (; g < ngroups; g += gstride) {
        const bhg_handle h = hn;
        const uint32_t i = g * 8 + r;
        const uint32_t gn = g + gstride;
        if (gn < ngroups && gn * 8 + r < n) hn = handles[gn * 8 + r];
        const bool valid = i < n;
        uint32_t st = BHG_ST_OK;
        bool inb = false;
        if (valid) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint32_t L = inb ? h.length : 0u;
        const uint64_t p = base + h.offset;
        const uint32_t m = inb ? (L + 127) / 128 : 1u;
        const uint32_t hl = L - 128 * (m - 1);
        const uint32_t jh = (m - 1) & 7;  // head lane
        const bool head = inb && j == jh;
        const int32_t q0 = (int32_t)(m - 1) - (int32_t)j;  // my last window
        // ---- loads: head (132 B from p & ~3) and first full window
        uint32_t hw[33], fw[33];
        const uint64_t ha = p & ~3ull;
        const uint32_t hsh = (uint32_t)(p & 3);
        if (head) {
            if (ha + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                    hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                }
                hw[32] = gld<uint32_t>(ha + 128);
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) hw[t] = ld32_safe(ha + 4 * t, end);
            }
        }
        // full windows of this lane in ascending order: q = qf, qf + 8, ..., q0 (qf >= 1)
        int32_t qf = q0 >= 1 ? (int32_t)(((uint32_t)q0 - 1) % 8 + 1) : 0;
        const uint64_t wsh_base = p + hl;  // start of window 1
        const uint32_t wsh = (uint32_t)(wsh_base & 3);
        auto load_win = [&](uint32_t *w, int32_t q) {
            const uint64_t a = (wsh_base + 128ull * (uint32_t)(q - 1)) & ~3ull;
            if (a + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const u32x4 v = gld<u32x4_a4>(a + 16 * t);
                    w[4 * t] = v.x; w[4 * t + 1] = v.y; w[4 * t + 2] = v.z; w[4 * t + 3] = v.w;
                }
                w[32] = gld<uint32_t>(a + 128);
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = ld32_safe(a + 4 * t, end);
            }
        };
        const bool hasw = inb && q0 >= 1;
        if (hasw) load_win(fw, qf);
        // ---- head CRC (from init) + header parse
        uint32_t acc = 0;
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;
        bool rvalid = false;
        if (head) {
            uint32_t c = 0xffffffffu;
            const uint32_t nw = hl >> 2;
            for (uint32_t t = 0; t < nw; t++) {
                uint32_t wv = 0, wn = 0;
#pragma unroll
                for (uint32_t u = 0; u < 32; u++) { wv = t == u ? hw[u] : wv; wn = t == u ? hw[u + 1] : wn; }
                c = crc.word(c, __builtin_amdgcn_alignbyte(wn, wv, hsh));
            }
            if (hl & 3) {
                uint32_t wv = 0, wn = 0;
#pragma unroll
                for (uint32_t u = 0; u < 32; u++) { wv = nw == u ? hw[u] : wv; wn = nw == u ? hw[u + 1] : wn; }
                c = crc.partial(c, __builtin_amdgcn_alignbyte(wn, wv, hsh), hl & 3);
            }
            acc = c;
            // header from registers (record bytes [0, 128) are in hw when L allows)
            uint32_t rw[14];
#pragma unroll
            for (int u = 0; u < 14; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            k = L >= 12 ? rw[0] : 0u;
            v = L >= 12 ? rw[1] : 0u;
            fn = L >= 12 ? rw[2] : 0u;
            rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (rvalid && k >= 8) {
                key_len = k - 8;
                if (key_len <= 36) {
                    uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                    for (uint32_t t = 3; t < 12; t++)
#pragma unroll
                        for (uint32_t b = 0; b < 4; b++) {
                            const uint32_t hn2 = (hh * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * b)) & 0xffu);
                            hh = 4 * (t - 3) + b < key_len ? hn2 : hh;
                        }
                    fnv = hh;
                    const uint32_t tb = 12 + key_len, tw = tb >> 2, ts = tb & 3;
                    uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                    for (uint32_t u = 3; u < 12; u++) {
                        a0 = tw == u ? rw[u] : a0;
                        a1 = tw == u ? rw[u + 1] : a1;
                        a2 = tw == u ? rw[u + 2] : a2;
                    }
                    trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                              ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        // ---- full windows
        if (hasw) {
            for (int32_t q = qf;; q += 8) {
                uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
                for (uint32_t t = 0; t < 8; t++)
#pragma unroll
                    for (uint32_t kk = 0; kk < 4; kk++) {
                        const uint32_t wi = 8 * kk + t;
                        c[kk] = crc.word(c[kk], __builtin_amdgcn_alignbyte(fw[wi + 1], fw[wi], wsh));
                    }
                // fold the 4 interleaved 32-B chains: V = Z96 c0 ^ Z64 c1 ^ Z32 c2 ^ c3, via Horner on Z32
                uint32_t V = zapply(ZS32, c[0]) ^ c[1];
                V = zapply(ZS32, V) ^ c[2];
                V = zapply(ZS32, V) ^ c[3];
                acc = zapply(Z, acc) ^ V;
                if (q + 8 > q0) break;
                load_win(fw, q + 8);
            }
        }
        // ---- move to the record end (Z_{128 j}) and reduce over the 8 lanes
        if (j & 1) acc = zapply(Z + 1024, acc);
        if (j & 2) acc = zapply(Z + 2048, acc);
        if (j & 4) acc = zapply(Z + 3072, acc);
        acc ^= __shfl_xor(acc, 1, 64);
        acc ^= __shfl_xor(acc, 2, 64);
        acc ^= __shfl_xor(acc, 4, 64);
        if (valid && j == jh) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) {
                const uint32_t crcv = crc_mask(~acc);
                if (rvalid) d = DescOutL{12, key_len, 12 + k, v, trailer, fn, fnv, crcv, BHG_ST_OK};
                else d = DescOutL{0, 0, 0, 0, 0, 0, 0, crcv, BHG_ST_RECORD_NIL};
            }
            store_descL(out + i, d);
        }
    }
}


// ============================================================== E10: two-phase tile (record lanes, then window lanes)
// A wave takes tiles of 64 consecutive handles.
// Phase 1, lane = record: handle, status, the record head [0, hl) (hl = L -
// 128 (m-1), 1..128 B) and the header / key / trailer prefix are loaded into
// registers; the head CRC (from 0xFFFFFFFF), the header checks, FNV-1 and the
// trailer are computed by all 64 lanes at once.
// Phase 2, 8 rounds of 8 records: lane (r, j) CRCs record 8s+r's full
// 128-B windows q = m-1-j, m-1-j-8, ... (>= 1; 132 B loads, a contiguous
// ~8.6 KB run per round), Horner-folds with Z_1024 starting from the head CRC
// (fetched from phase 1) on lane j == (m-1) % 8, shifts by Z_{128 j}, and
// the 8 lanes xor-reduce.  The next round's windows are loaded before the
// current round is absorbed.
template <int WPB, int R, int MODE>
__global__ __launch_bounds__(64 * WPB) void k_tile(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Lds<R>::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[5 * 1024];  // Z1024, Z128, Z256, Z512, Z32
    Crc4Lds<R>::fill(T);
    for (uint32_t t = threadIdx.x; t < 5 * 1024; t += 64 * WPB) Z[t] = gz[t];
    __syncthreads();
    const uint32_t *ZS32 = Z + 4096;
    const Crc4Lds<R> crc(T);
    auto zapply = [&](const uint32_t *Zt, uint32_t c) {
        return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
    };
    const uint32_t lane = threadIdx.x & 63, rr = lane >> 3, j = lane & 7;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t tstride = gridDim.x * WPB;
    uint32_t tile = blockIdx.x * WPB + (threadIdx.x >> 6);
    bhg_handle hn = {0, 0, 0};
    if (tile < ntiles && tile * 64 + lane < n) hn = handles[tile * 64 + lane];
    for (; tile < ntiles; tile += tstride) {
        // ---------------- phase 1: lane = record
        const bhg_handle h = hn;
        const uint32_t i = tile * 64 + lane;
        {
            const uint32_t tn = tile + tstride;
            if (tn < ntiles && tn * 64 + lane < n) hn = handles[tn * 64 + lane];
        }
        const bool valid = i < n;
        uint32_t st = BHG_ST_OK;
        bool inb = false;
        if (valid) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint32_t L = inb ? h.length : 0u;
        const uint64_t p = base + h.offset;
        const uint32_t m = inb ? (L + 127) / 128 : 1u;
        const uint32_t hl = L - 128 * (m - 1);
        uint32_t hw[33];
        const uint64_t ha = p & ~3ull;
        const uint32_t hsh = (uint32_t)(p & 3);
        if (inb) {
            if (ha + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                    hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                }
                if (hl > 60) {
#pragma unroll
                    for (int t = 4; t < 8; t++) {
                        const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                        hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                    }
                    hw[32] = gld<uint32_t>(ha + 128);
                } else {
#pragma unroll
                    for (int t = 16; t < 33; t++) hw[t] = 0;
                }
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) hw[t] = ld32_safe(ha + 4 * t, end);
            }
        }
        uint32_t hcrc = 0xffffffffu;
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;
        bool rvalid = false;
        if (inb) {
            const uint32_t nw = hl >> 2;
#pragma unroll
            for (uint32_t u = 0; u < 32; u++)
                if (u < nw) hcrc = crc.word(hcrc, __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh));
            if (hl & 3) {
                uint32_t wv = 0, wn = 0;
#pragma unroll
                for (uint32_t u = 0; u < 32; u++) { wv = nw == u ? hw[u] : wv; wn = nw == u ? hw[u + 1] : wn; }
                hcrc = crc.partial(hcrc, __builtin_amdgcn_alignbyte(wn, wv, hsh), hl & 3);
            }
            uint32_t rw[14];
#pragma unroll
            for (int u = 0; u < 14; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            k = L >= 12 ? rw[0] : 0u;
            v = L >= 12 ? rw[1] : 0u;
            fn = L >= 12 ? rw[2] : 0u;
            rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (rvalid && k >= 8) {
                key_len = k - 8;
                if (key_len <= 36) {
                    uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                    for (uint32_t t = 3; t < 12; t++)
#pragma unroll
                        for (uint32_t b = 0; b < 4; b++) {
                            const uint32_t hn2 = (hh * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * b)) & 0xffu);
                            hh = 4 * (t - 3) + b < key_len ? hn2 : hh;
                        }
                    fnv = hh;
                    const uint32_t tb = 12 + key_len, tw = tb >> 2, ts = tb & 3;
                    uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                    for (uint32_t u = 3; u < 12; u++) {
                        a0 = tw == u ? rw[u] : a0;
                        a1 = tw == u ? rw[u + 1] : a1;
                        a2 = tw == u ? rw[u + 2] : a2;
                    }
                    trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                              ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        // ---------------- phase 2: 8 rounds, lane (rr, j) on record 8s + rr
        uint32_t mycrc = 0;
        uint32_t fw[2][33];
        auto rinfo = [&](uint32_t s, uint64_t &wb, uint32_t &mm, int32_t &qf, int32_t &q0, bool &hasw) {
            const uint32_t src_l = 8 * s + rr;
            const uint32_t Lr = __shfl(L, src_l, 64);
            const uint64_t pr = shfl64(p, src_l);
            mm = __shfl(m, src_l, 64);
            const uint32_t hlr = Lr - 128 * (mm - 1);
            wb = pr + hlr;
            q0 = (int32_t)(mm - 1) - (int32_t)j;
            hasw = Lr != 0 && q0 >= 1;
            qf = q0 >= 1 ? (int32_t)(((uint32_t)q0 - 1) % 8 + 1) : 0;
        };
        auto load_win = [&](uint32_t *w, uint64_t wb, int32_t q) {
            const uint64_t a = (wb + 128ull * (uint32_t)(q - 1)) & ~3ull;
            if (a + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const u32x4 x = gld<u32x4_a4>(a + 16 * t);
                    w[4 * t] = x.x; w[4 * t + 1] = x.y; w[4 * t + 2] = x.z; w[4 * t + 3] = x.w;
                }
                w[32] = gld<uint32_t>(a + 128);
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = ld32_safe(a + 4 * t, end);
            }
        };
        uint64_t wb;
        uint32_t mm;
        int32_t qf, q0;
        bool hasw;
        rinfo(0, wb, mm, qf, q0, hasw);
        if (hasw) load_win(fw[0], wb, qf);
#pragma unroll
        for (uint32_t s = 0; s < 8; s++) {
            const uint32_t cb = s & 1;
            const uint64_t wb_c = wb;
            const uint32_t mm_c = mm;
            const int32_t qf_c = qf, q0_c = q0;
            const bool hasw_c = hasw;
            if (s + 1 < 8) {
                rinfo(s + 1, wb, mm, qf, q0, hasw);
                if (hasw) load_win(fw[cb ^ 1], wb, qf);
            }
            const uint32_t hc = __shfl(hcrc, 8 * s + rr, 64);
            uint32_t acc = (j == ((mm_c - 1) & 7)) ? hc : 0u;
            if (hasw_c) {
                const uint32_t wsh = (uint32_t)(wb_c & 3);
                for (int32_t q = qf_c;; q += 8) {
                    uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
                    for (uint32_t t = 0; t < 8; t++)
#pragma unroll
                        for (uint32_t kk = 0; kk < 4; kk++) {
                            const uint32_t wi = 8 * kk + t;
                            c[kk] = crc.word(c[kk], __builtin_amdgcn_alignbyte(fw[cb][wi + 1], fw[cb][wi], wsh));
                        }
                    uint32_t V = zapply(ZS32, c[0]) ^ c[1];
                    V = zapply(ZS32, V) ^ c[2];
                    V = zapply(ZS32, V) ^ c[3];
                    acc = zapply(Z, acc) ^ V;
                    if (q + 8 > q0_c) break;
                    load_win(fw[cb], wb_c, q + 8);
                }
            }
            if (j & 1) acc = zapply(Z + 1024, acc);
            if (j & 2) acc = zapply(Z + 2048, acc);
            if (j & 4) acc = zapply(Z + 3072, acc);
            acc ^= __shfl_xor(acc, 1, 64);
            acc ^= __shfl_xor(acc, 2, 64);
            acc ^= __shfl_xor(acc, 4, 64);
            // record 8s + rr's total is on lanes 8 rr .. 8 rr + 7; lane l = 8 s + r takes lane 8 r
            const uint32_t got = __shfl(acc, 8 * (lane & 7), 64);
            if ((lane >> 3) == s) mycrc = got;
        }
        if (valid) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) {
                const uint32_t crcv = crc_mask(~mycrc);
                if (rvalid) d = DescOutL{12, key_len, 12 + k, v, trailer, fn, fnv, crcv, BHG_ST_OK};
                else d = DescOutL{0, 0, 0, 0, 0, 0, 0, crcv, BHG_ST_RECORD_NIL};
            }
            store_descL(out + i, d);
        }
    }
}

template <int WPB, class Tab, int MODE>
__global__ __launch_bounds__(64 * WPB) void k_tile2(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Tab::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[5 * 1024];  // Z1024, Z128, Z256, Z512, Z32
    Tab::fill(T);
    for (uint32_t t = threadIdx.x; t < 5 * 1024; t += 64 * WPB) Z[t] = gz[t];
    __syncthreads();
    const uint32_t *ZS32 = Z + 4096;
    const Tab crc(T);
    auto zapply = [&](const uint32_t *Zt, uint32_t c) {
        return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
    };
    const uint32_t lane = threadIdx.x & 63, rr = lane >> 3, j = lane & 7;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t tstride = gridDim.x * WPB;
    uint32_t tile = blockIdx.x * WPB + (threadIdx.x >> 6);
    bhg_handle hn = {0, 0, 0};
    if (tile < ntiles && tile * 64 + lane < n) hn = handles[tile * 64 + lane];
    for (; tile < ntiles; tile += tstride) {
        // ---------------- phase 1: lane = record
        const bhg_handle h = hn;
        const uint32_t i = tile * 64 + lane;
        {
            const uint32_t tn = tile + tstride;
            if (tn < ntiles && tn * 64 + lane < n) hn = handles[tn * 64 + lane];
        }
        const bool valid = i < n;
        uint32_t st = BHG_ST_OK;
        bool inb = false;
        if (valid) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint32_t L = inb ? h.length : 0u;
        const uint64_t p = base + h.offset;
        const uint32_t m = inb ? (L + 127) / 128 : 1u;
        const uint32_t hl = L - 128 * (m - 1);
        uint32_t hw[33];
        const uint64_t ha = p & ~3ull;
        const uint32_t hsh = (uint32_t)(p & 3);
        if (inb && (MODE & 8)) {  // diag: no phase-1 loads (synthetic header of a valid C2 record)
#pragma unroll
            for (int t = 0; t < 33; t++) hw[t] = t == 0 ? 40u : t == 1 ? 1024u : (uint32_t)p + t;
        } else if (inb) {
            if (ha + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                    hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                }
                if (hl > 60) {
#pragma unroll
                    for (int t = 4; t < 8; t++) {
                        const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                        hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                    }
                    hw[32] = gld<uint32_t>(ha + 128);
                } else {
#pragma unroll
                    for (int t = 16; t < 33; t++) hw[t] = 0;
                }
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) hw[t] = ld32_safe(ha + 4 * t, end);
            }
        }
        uint32_t hcrc = 0xffffffffu;
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;
        bool rvalid = false;
        if (inb) {
            const uint32_t nw = hl >> 2;
#pragma unroll
            for (uint32_t u = 0; u < 32; u++)
                if (u < nw) hcrc = crc.word(hcrc, __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh));
            if (hl & 3) {
                uint32_t wv = 0, wn = 0;
#pragma unroll
                for (uint32_t u = 0; u < 32; u++) { wv = nw == u ? hw[u] : wv; wn = nw == u ? hw[u + 1] : wn; }
                hcrc = crc.partial(hcrc, __builtin_amdgcn_alignbyte(wn, wv, hsh), hl & 3);
            }
            uint32_t rw[14];
#pragma unroll
            for (int u = 0; u < 14; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            k = L >= 12 ? rw[0] : 0u;
            v = L >= 12 ? rw[1] : 0u;
            fn = L >= 12 ? rw[2] : 0u;
            rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (rvalid && k >= 8) {
                key_len = k - 8;
                if (key_len <= 36) {
                    uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                    for (uint32_t t = 3; t < 12; t++)
#pragma unroll
                        for (uint32_t b = 0; b < 4; b++) {
                            const uint32_t hn2 = (hh * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * b)) & 0xffu);
                            hh = 4 * (t - 3) + b < key_len ? hn2 : hh;
                        }
                    fnv = hh;
                    const uint32_t tb = 12 + key_len, tw = tb >> 2, ts = tb & 3;
                    uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                    for (uint32_t u = 3; u < 12; u++) {
                        a0 = tw == u ? rw[u] : a0;
                        a1 = tw == u ? rw[u + 1] : a1;
                        a2 = tw == u ? rw[u + 2] : a2;
                    }
                    trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                              ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        // ---------------- phase 2: 8 rounds, lane (rr, j) on record 8s + rr
        uint32_t mycrc = 0;
        uint32_t fw[2][33];  // MODE & 1: next round loaded after this round is absorbed
        auto rinfo = [&](uint32_t s, uint64_t &wb, uint32_t &mm, int32_t &qf, int32_t &q0, bool &hasw) {
            const uint32_t src_l = 8 * s + rr;
            const uint32_t Lr = __shfl(L, src_l, 64);
            const uint64_t pr = shfl64(p, src_l);
            mm = __shfl(m, src_l, 64);
            const uint32_t hlr = Lr - 128 * (mm - 1);
            wb = pr + hlr;
            q0 = (int32_t)(mm - 1) - (int32_t)j;
            hasw = Lr != 0 && q0 >= 1;
            qf = q0 >= 1 ? (int32_t)(((uint32_t)q0 - 1) % 8 + 1) : 0;
        };
        auto load_win = [&](uint32_t *w, uint64_t wb, int32_t q) {
            const uint64_t a = (wb + 128ull * (uint32_t)(q - 1)) & ~3ull;
            if (MODE & 2) {  // diag: compute only
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = (uint32_t)a * 0x9e3779b9u + t;
            } else if (a + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const u32x4 x = gld<u32x4_a4>(a + 16 * t);
                    w[4 * t] = x.x; w[4 * t + 1] = x.y; w[4 * t + 2] = x.z; w[4 * t + 3] = x.w;
                }
                w[32] = gld<uint32_t>(a + 128);
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = ld32_safe(a + 4 * t, end);
            }
        };
        uint64_t wb;
        uint32_t mm;
        int32_t qf, q0;
        bool hasw;
        rinfo(0, wb, mm, qf, q0, hasw);
        if (hasw) load_win(fw[0], wb, qf);
#pragma unroll
        for (uint32_t s = 0; s < 8; s++) {
            const uint32_t cb = (MODE & 1) ? 0u : (s & 1);
            const uint64_t wb_c = wb;
            const uint32_t mm_c = mm;
            const int32_t qf_c = qf, q0_c = q0;
            const bool hasw_c = hasw;
            if (!(MODE & 1) && s + 1 < 8) {
                rinfo(s + 1, wb, mm, qf, q0, hasw);
                if (hasw) load_win(fw[cb ^ 1], wb, qf);
            }
            const uint32_t hc = __shfl(hcrc, 8 * s + rr, 64);
            uint32_t acc = (j == ((mm_c - 1) & 7)) ? hc : 0u;
            if (hasw_c) {
                const uint32_t wsh = (uint32_t)(wb_c & 3);
                for (int32_t q = qf_c;; q += 8) {
                    uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
                    for (uint32_t t = 0; t < 8; t++)
#pragma unroll
                        for (uint32_t kk = 0; kk < 4; kk++) {
                            const uint32_t wi = 8 * kk + t;
                            const uint32_t wv = __builtin_amdgcn_alignbyte(fw[cb][wi + 1], fw[cb][wi], wsh);
                            c[kk] = (MODE & 4) ? (((c[kk] << 1) | (c[kk] >> 31)) ^ wv) : crc.word(c[kk], wv);
                        }
                    uint32_t V = zapply(ZS32, c[0]) ^ c[1];
                    V = zapply(ZS32, V) ^ c[2];
                    V = zapply(ZS32, V) ^ c[3];
                    acc = zapply(Z, acc) ^ V;
                    if (q + 8 > q0_c) break;
                    load_win(fw[cb], wb_c, q + 8);
                }
            }
            if ((MODE & 1) && s + 1 < 8) {
                rinfo(s + 1, wb, mm, qf, q0, hasw);
                if (hasw) load_win(fw[0], wb, qf);
            }
            if (j & 1) acc = zapply(Z + 1024, acc);
            if (j & 2) acc = zapply(Z + 2048, acc);
            if (j & 4) acc = zapply(Z + 3072, acc);
            acc ^= __shfl_xor(acc, 1, 64);
            acc ^= __shfl_xor(acc, 2, 64);
            acc ^= __shfl_xor(acc, 4, 64);
            // record 8s + rr's total is on lanes 8 rr .. 8 rr + 7; lane l = 8 s + r takes lane 8 r
            const uint32_t got = __shfl(acc, 8 * (lane & 7), 64);
            if ((lane >> 3) == s) mycrc = got;
        }
        if (valid) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) {
                const uint32_t crcv = crc_mask(~mycrc);
                if (rvalid) d = DescOutL{12, key_len, 12 + k, v, trailer, fn, fnv, crcv, BHG_ST_OK};
                else d = DescOutL{0, 0, 0, 0, 0, 0, 0, crcv, BHG_ST_RECORD_NIL};
            }
            store_descL(out + i, d);
        }
    }
}

template <int WPB, class Tab, int MODE, int PD>
__global__ __launch_bounds__(64 * WPB) void k_tile3(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Tab::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[5 * 1024];  // Z1024, Z128, Z256, Z512, Z32
    Tab::fill(T);
    for (uint32_t t = threadIdx.x; t < 5 * 1024; t += 64 * WPB) Z[t] = gz[t];
    __syncthreads();
    const uint32_t *ZS32 = Z + 4096;
    const Tab crc(T);
    auto zapply = [&](const uint32_t *Zt, uint32_t c) {
        return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
    };
    const uint32_t lane = threadIdx.x & 63, rr = lane >> 3, j = lane & 7;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t tstride = gridDim.x * WPB;
    uint32_t tile = blockIdx.x * WPB + (threadIdx.x >> 6);
    bhg_handle hn = {0, 0, 0};
    if (tile < ntiles && tile * 64 + lane < n) hn = handles[tile * 64 + lane];
    for (; tile < ntiles; tile += tstride) {
        // ---------------- phase 1: lane = record
        const bhg_handle h = hn;
        const uint32_t i = tile * 64 + lane;
        {
            const uint32_t tn = tile + tstride;
            if (tn < ntiles && tn * 64 + lane < n) hn = handles[tn * 64 + lane];
        }
        const bool valid = i < n;
        uint32_t st = BHG_ST_OK;
        bool inb = false;
        if (valid) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint32_t L = inb ? h.length : 0u;
        const uint64_t p = base + h.offset;
        const uint32_t m = inb ? (L + 127) / 128 : 1u;
        const uint32_t hl = L - 128 * (m - 1);
        uint32_t hw[33];
        const uint64_t ha = p & ~3ull;
        const uint32_t hsh = (uint32_t)(p & 3);
        if (inb && (MODE & 8)) {  // diag: no phase-1 loads (synthetic header of a valid C2 record)
#pragma unroll
            for (int t = 0; t < 33; t++) hw[t] = t == 0 ? 40u : t == 1 ? 1024u : (uint32_t)p + t;
        } else if (inb) {
            if (ha + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                    hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                }
                if (hl > 60) {
#pragma unroll
                    for (int t = 4; t < 8; t++) {
                        const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                        hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                    }
                    hw[32] = gld<uint32_t>(ha + 128);
                } else {
#pragma unroll
                    for (int t = 16; t < 33; t++) hw[t] = 0;
                }
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) hw[t] = ld32_safe(ha + 4 * t, end);
            }
        }
        uint32_t hcrc = 0xffffffffu;
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;
        bool rvalid = false;
        if (inb) {
            const uint32_t nw = hl >> 2;
#pragma unroll
            for (uint32_t u = 0; u < 32; u++)
                if (u < nw) hcrc = crc.word(hcrc, __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh));
            if (hl & 3) {
                uint32_t wv = 0, wn = 0;
#pragma unroll
                for (uint32_t u = 0; u < 32; u++) { wv = nw == u ? hw[u] : wv; wn = nw == u ? hw[u + 1] : wn; }
                hcrc = crc.partial(hcrc, __builtin_amdgcn_alignbyte(wn, wv, hsh), hl & 3);
            }
            uint32_t rw[14];
#pragma unroll
            for (int u = 0; u < 14; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            k = L >= 12 ? rw[0] : 0u;
            v = L >= 12 ? rw[1] : 0u;
            fn = L >= 12 ? rw[2] : 0u;
            rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (rvalid && k >= 8) {
                key_len = k - 8;
                if (key_len <= 36) {
                    uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                    for (uint32_t t = 3; t < 12; t++)
#pragma unroll
                        for (uint32_t b = 0; b < 4; b++) {
                            const uint32_t hn2 = (hh * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * b)) & 0xffu);
                            hh = 4 * (t - 3) + b < key_len ? hn2 : hh;
                        }
                    fnv = hh;
                    const uint32_t tb = 12 + key_len, tw = tb >> 2, ts = tb & 3;
                    uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                    for (uint32_t u = 3; u < 12; u++) {
                        a0 = tw == u ? rw[u] : a0;
                        a1 = tw == u ? rw[u + 1] : a1;
                        a2 = tw == u ? rw[u + 2] : a2;
                    }
                    trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                              ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        // ---------------- phase 2: 8 rounds, lane (rr, j) on record 8s + rr
        uint32_t mycrc = 0;
        auto rinfo = [&](uint32_t s, uint64_t &wb, uint32_t &mm, int32_t &qf, int32_t &q0, bool &hasw) {
            const uint32_t src_l = 8 * s + rr;
            const uint32_t Lr = __shfl(L, src_l, 64);
            const uint64_t pr = shfl64(p, src_l);
            mm = __shfl(m, src_l, 64);
            const uint32_t hlr = Lr - 128 * (mm - 1);
            wb = pr + hlr;
            q0 = (int32_t)(mm - 1) - (int32_t)j;
            hasw = Lr != 0 && q0 >= 1;
            qf = q0 >= 1 ? (int32_t)(((uint32_t)q0 - 1) % 8 + 1) : 0;
        };
        auto load_win = [&](uint32_t *w, uint64_t wb, int32_t q) {
            const uint64_t a = (wb + 128ull * (uint32_t)(q - 1)) & ~3ull;
            if (MODE & 2) {  // diag: compute only
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = (uint32_t)a * 0x9e3779b9u + t;
            } else if (a + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const u32x4 x = gld<u32x4_a4>(a + 16 * t);
                    w[4 * t] = x.x; w[4 * t + 1] = x.y; w[4 * t + 2] = x.z; w[4 * t + 3] = x.w;
                }
                w[32] = gld<uint32_t>(a + 128);
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = ld32_safe(a + 4 * t, end);
            }
        };
        constexpr int NB = PD + 1;
        uint32_t fwb[NB][33];
        uint64_t wbA[NB];
        uint32_t mmA[NB];
        int32_t qfA[NB], q0A[NB];
        bool hasA[NB];
#pragma unroll
        for (int s0 = 0; s0 < PD; s0++) {
            rinfo(s0, wbA[s0], mmA[s0], qfA[s0], q0A[s0], hasA[s0]);
            if (hasA[s0]) load_win(fwb[s0], wbA[s0], qfA[s0]);
        }
#pragma unroll
        for (uint32_t s = 0; s < 8; s++) {
            const int cb = s % NB;
            if (s + PD < 8) {
                const int nb = (s + PD) % NB;
                rinfo(s + PD, wbA[nb], mmA[nb], qfA[nb], q0A[nb], hasA[nb]);
                if (hasA[nb]) load_win(fwb[nb], wbA[nb], qfA[nb]);
            }
            const uint64_t wb_c = wbA[cb];
            const uint32_t mm_c = mmA[cb];
            const int32_t qf_c = qfA[cb], q0_c = q0A[cb];
            const bool hasw_c = hasA[cb];
            const uint32_t hc = __shfl(hcrc, 8 * s + rr, 64);
            uint32_t acc = (j == ((mm_c - 1) & 7)) ? hc : 0u;
            if (hasw_c) {
                const uint32_t wsh = (uint32_t)(wb_c & 3);
                for (int32_t q = qf_c;; q += 8) {
                    uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
                    for (uint32_t t = 0; t < 8; t++)
#pragma unroll
                        for (uint32_t kk = 0; kk < 4; kk++) {
                            const uint32_t wi = 8 * kk + t;
                            const uint32_t wv = __builtin_amdgcn_alignbyte(fwb[cb][wi + 1], fwb[cb][wi], wsh);
                            c[kk] = (MODE & 4) ? (((c[kk] << 1) | (c[kk] >> 31)) ^ wv) : crc.word(c[kk], wv);
                        }
                    uint32_t V = zapply(ZS32, c[0]) ^ c[1];
                    V = zapply(ZS32, V) ^ c[2];
                    V = zapply(ZS32, V) ^ c[3];
                    acc = zapply(Z, acc) ^ V;
                    if (q + 8 > q0_c) break;
                    load_win(fwb[cb], wb_c, q + 8);
                }
            }
            if (j & 1) acc = zapply(Z + 1024, acc);
            if (j & 2) acc = zapply(Z + 2048, acc);
            if (j & 4) acc = zapply(Z + 3072, acc);
            acc ^= __shfl_xor(acc, 1, 64);
            acc ^= __shfl_xor(acc, 2, 64);
            acc ^= __shfl_xor(acc, 4, 64);
            // record 8s + rr's total is on lanes 8 rr .. 8 rr + 7; lane l = 8 s + r takes lane 8 r
            const uint32_t got = __shfl(acc, 8 * (lane & 7), 64);
            if ((lane >> 3) == s) mycrc = got;
        }
        if (valid) {
            DescOutL d = {0, 0, 0, 0, 0, 0, 0, 0, st};
            if (inb) {
                const uint32_t crcv = crc_mask(~mycrc);
                if (rvalid) d = DescOutL{12, key_len, 12 + k, v, trailer, fn, fnv, crcv, BHG_ST_OK};
                else d = DescOutL{0, 0, 0, 0, 0, 0, 0, crcv, BHG_ST_RECORD_NIL};
            }
            if (!(MODE & 16)) store_descL(out + i, d);
            else if (d.crc == 0x12345678u) reinterpret_cast<uint32_t *>(out)[lane] = d.fnv1;
        }
    }
}


__device__ __forceinline__ uint32_t zapply4(const uint32_t *Zt, uint32_t c) {
    return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
}
// E11: tile kernel, one window per lane per round, PD rounds of loads in flight
template <int WPB, int PD, int MODE>
__global__ __launch_bounds__(64 * WPB) void k_tile4(const uint8_t *__restrict__ src, uint64_t src_len,
                                                          const bhg_handle *__restrict__ handles, uint32_t n,
                                                          bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[5 * 1024];  // Z1024, Z128, Z256, Z512, Z32
    Crc4Perm::fill(T);
    for (uint32_t t = threadIdx.x; t < 5 * 1024; t += 64 * WPB) Z[t] = gz[t];
    __syncthreads();
    const uint32_t *Z32 = Z + 4096;
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63, rr = lane >> 3, j = lane & 7;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t tstride = gridDim.x * WPB;
    uint32_t tile = blockIdx.x * WPB + (threadIdx.x >> 6);
    bhg_handle hn = {0, 0, 0};
    if (tile < ntiles && tile * 64 + lane < n) hn = handles[tile * 64 + lane];
    for (; tile < ntiles; tile += tstride) {
        // ---------------- phase 1: lane = record (Reader.readData's checks, readRecord, readKV)
        const bhg_handle h = hn;
        const uint32_t i = tile * 64 + lane;
        {
            const uint32_t tn = tile + tstride;
            if (tn < ntiles && tn * 64 + lane < n) hn = handles[tn * 64 + lane];
        }
        const bool valid = i < n;
        uint32_t st = BHG_ST_OK;
        bool inb = false;
        if (valid) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;                    // reader.go:234-236
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset)
                st = BHG_ST_INCOMPLETE;                                       // reader.go:251-258
            else inb = true;
        }
        const uint32_t L = inb ? h.length : 0u;
        const uint64_t p = base + h.offset;
        const uint32_t m = inb ? (L + 127) / 128 : 1u;
        const uint32_t hl = L - 128 * (m - 1);
        uint32_t hw[33];
        const uint64_t ha = p & ~3ull;
        const uint32_t hsh = (uint32_t)(p & 3);
        if (inb) {
            if (ha + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                    hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                }
                if (hl > 60) {
#pragma unroll
                    for (int t = 4; t < 8; t++) {
                        const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                        hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                    }
                    hw[32] = gld<uint32_t>(ha + 128);
                } else {
#pragma unroll
                    for (int t = 16; t < 33; t++) hw[t] = 0;
                }
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) hw[t] = ld32_safe(ha + 4 * t, end);
            }
        }
        uint32_t hcrc = 0xffffffffu;  // crc.New: Go's crc32.Update starts from ^0
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;       // InternalKeyKindInvalid when ikeySize < 8
        bool rvalid = false;
        if (inb) {
            const uint32_t nw = hl >> 2;
#pragma unroll
            for (uint32_t u = 0; u < 32; u++)
                if (u < nw) hcrc = crc.word(hcrc, __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh));
            if (hl & 3) {
                uint32_t wv = 0, wn = 0;
#pragma unroll
                for (uint32_t u = 0; u < 32; u++) {
                    wv = nw == u ? hw[u] : wv;
                    wn = nw == u ? hw[u + 1] : wn;
                }
                hcrc = crc.partial(hcrc, __builtin_amdgcn_alignbyte(wn, wv, hsh), hl & 3);
            }
            uint32_t rw[14];
#pragma unroll
            for (int u = 0; u < 14; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            // readRecordHeader (block2.go:31-36) + readRecord's length check (:57-66)
            k = L >= 12 ? rw[0] : 0u;
            v = L >= 12 ? rw[1] : 0u;
            fn = L >= 12 ? rw[2] : 0u;
            rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (rvalid && k >= 8) {  // readKV / DecodeInternalKey (block2.go:38-55)
                key_len = k - 8;
                if (key_len <= 36) {
                    uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                    for (uint32_t t = 3; t < 12; t++)
#pragma unroll
                        for (uint32_t b = 0; b < 4; b++) {
                            const uint32_t h2 = (hh * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * b)) & 0xffu);
                            hh = 4 * (t - 3) + b < key_len ? h2 : hh;
                        }
                    fnv = hh;
                    const uint32_t tb = 12 + key_len, tw = tb >> 2, ts = tb & 3;
                    uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                    for (uint32_t u = 3; u <= 12; u++) {  // tb <= 48: the trailer ends by byte 56 = rw[13]
                        a0 = tw == u ? rw[u] : a0;
                        a1 = tw == u ? rw[u + 1] : a1;
                        if (u + 2 < 14) a2 = tw == u ? rw[u + 2] : a2;  // tw == 12 only with ts == 0
                    }
                    trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                              ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        // ---------------- phase 2: 8 rounds, one window per lane per round, PD rounds in flight
        const bool big = inb && m > 9;  // more than one window per lane: slow path below
        uint32_t mycrc = 0;
        constexpr int NB = PD + 1;
        uint32_t fw[NB][33];
        uint64_t wa[NB];
        bool hw_[NB];
        uint32_t hsel[NB];
        auto rinfo = [&](uint32_t s, uint64_t &a, bool &has, uint32_t &hs) {
            const uint32_t sl = 8 * s + rr;
            const uint32_t Lr = __shfl(L, sl, 64);
            const uint64_t pr = shfl64(p, sl);
            const uint32_t mr = __shfl(m, sl, 64);
            const int32_t q = (int32_t)(mr - 1) - (int32_t)j;  // my window (>= 1)
            has = Lr != 0 && mr <= 9 && q >= 1;
            a = pr + (Lr - 128 * (mr - 1)) + 128ull * (uint32_t)(q - 1);
            hs = (mr <= 9 && j == ((mr - 1) & 7)) ? 1u : 0u;
        };
        auto load_win = [&](uint32_t *w, uint64_t a0) {
            const uint64_t a = a0 & ~3ull;
            if (MODE & 2) {
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = (uint32_t)a * 0x9e3779b9u + t;
            } else if (a + 132 <= end) {
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const u32x4 x = gld<u32x4_a4>(a + 16 * t);
                    w[4 * t] = x.x; w[4 * t + 1] = x.y; w[4 * t + 2] = x.z; w[4 * t + 3] = x.w;
                }
                w[32] = gld<uint32_t>(a + 128);
            } else {
#pragma unroll
                for (int t = 0; t < 33; t++) w[t] = ld32_safe(a + 4 * t, end);
            }
        };
#pragma unroll
        for (int s0 = 0; s0 < PD; s0++) {
            rinfo(s0, wa[s0], hw_[s0], hsel[s0]);
            if (hw_[s0]) load_win(fw[s0], wa[s0]);
        }
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const int cb = s % NB;
            if (s + PD < 8) {
                const int nb = (s + PD) % NB;
                rinfo(s + PD, wa[nb], hw_[nb], hsel[nb]);
                if (hw_[nb]) load_win(fw[nb], wa[nb]);
            }
            const uint32_t hc = __shfl(hcrc, 8 * s + rr, 64);
            uint32_t acc = hsel[cb] ? hc : 0u;
            if (hw_[cb]) {
                const uint32_t wsh = (uint32_t)(wa[cb] & 3);
                uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
                for (uint32_t t = 0; t < 8; t++)
#pragma unroll
                    for (uint32_t kk = 0; kk < 4; kk++) {
                        const uint32_t wi = 8 * kk + t;
                        const uint32_t wv = __builtin_amdgcn_alignbyte(fw[cb][wi + 1], fw[cb][wi], wsh);
                        c[kk] = (MODE & 4) ? (((c[kk] << 1) | (c[kk] >> 31)) ^ wv) : crc.word(c[kk], wv);
                    }
                uint32_t V = zapply4(Z32, c[0]) ^ c[1];
                V = zapply4(Z32, V) ^ c[2];
                V = zapply4(Z32, V) ^ c[3];
                acc = zapply4(Z, acc) ^ V;
            }
            if (j & 1) acc = zapply4(Z + 1024, acc);
            if (j & 2) acc = zapply4(Z + 2048, acc);
            if (j & 4) acc = zapply4(Z + 3072, acc);
            acc ^= __shfl_xor(acc, 1, 64);
            acc ^= __shfl_xor(acc, 2, 64);
            acc ^= __shfl_xor(acc, 4, 64);
            const uint32_t got = __shfl(acc, 8 * (lane & 7), 64);
            if ((lane >> 3) == (uint32_t)s) mycrc = got;
        }
        if (big) mycrc = crc_range_a<8, Crc4Perm, true>(crc, 0xffffffffu, p, L, end);
        if (valid) {
            uint32_t dk = 0, dkl = 0, dvo = 0, dvl = 0, dfn = 0, dfnv = 0, dcrc = 0, dst = st;
            uint64_t dtr = 0;
            if (inb) {
                dcrc = crc_mask(~mycrc);  // crc.go:31-33
                if (rvalid) {
                    dk = 12; dkl = key_len; dvo = 12 + k; dvl = v;  // noCompressor.Decode: zero-copy view
                    dtr = trailer; dfn = fn; dfnv = fnv;
                    
                } else {
                    dst = BHG_ST_RECORD_NIL;  // ErrBhReadRecordNil
                }
            }
            if (MODE & 16) { if (dcrc == 0x12345678u) reinterpret_cast<uint32_t *>(out)[lane] = dfnv; continue; }
            uint2 *o = reinterpret_cast<uint2 *>(out + i);
            o[0] = make_uint2(dk, dkl);
            o[1] = make_uint2(dvo, dvl);
            o[2] = make_uint2((uint32_t)dtr, (uint32_t)(dtr >> 32));
            o[3] = make_uint2(dfn, dfnv);
            o[4] = make_uint2(dcrc, dst);
        }
    }
}


// ============================================================== launchers
static int g_cus = 256;
constexpr uint32_t kLabShiftSets = 3;  // CH = 64, 128, 256
constexpr uint32_t kLabNB = 6;
constexpr size_t kLabBraidOff = kLabShiftSets * kLabNB * 1024;        // words
constexpr size_t kLabBraidSet = 6 * 1024;                                // braid table + up to 5 tree levels
constexpr size_t kLabZ128Off = kLabBraidOff + 5 * kLabBraidSet;
constexpr size_t kLabPlainOff = kLabZ128Off + 1024;   // plain slice-by-4 then Z128 (sweep2 layout)
constexpr size_t kLabL5Off = kLabPlainOff + 2048;     // plain slice-by-4, Z4..Z128
constexpr size_t kLabStageOff = kLabL5Off + 7 * 1024;  // Z32, Z1024, Z128, Z256, Z512 (k_stage, S = 8)
constexpr size_t kLabWinOff = kLabStageOff + 5 * 1024;  // Z1024, Z128, Z256, Z512, Z32 (k_win)
constexpr size_t kLabTabBytes = (kLabWinOff + 5 * 1024) * 4;
static void lab_init_tables(uint32_t *d) {
    std::vector<uint32_t> h(kLabTabBytes / 4);
    const uint32_t chs[3] = {64, 128, 256};
    for (uint32_t s = 0; s < 3; s++)
        for (uint32_t b = 0; b < kLabNB; b++) crc32c_shift_table((uint64_t)chs[s] << b, &h[(s * kLabNB + b) * 1024]);
    for (uint32_t lg = 1; lg <= 5; lg++) {
        const uint32_t G = 1u << lg;
        uint32_t *o = &h[kLabBraidOff + (lg - 1) * kLabBraidSet];
        crc32c_braid_table(4ull * (G - 1), o);
        for (uint32_t s = 0; s < lg; s++) gf2_table(crc32c_unzero_bytes(4ull << s), o + 1024 * (1 + s));
    }
    crc32c_shift_table(128, &h[kLabZ128Off]);
    for (uint32_t k = 0; k < 4; k++)
        for (uint32_t b = 0; b < 256; b++) h[kLabPlainOff + k * 256 + b] = crc32c_tk(k, b);
    crc32c_shift_table(128, &h[kLabPlainOff + 1024]);
    for (uint32_t k = 0; k < 4; k++)
        for (uint32_t b = 0; b < 256; b++) h[kLabL5Off + k * 256 + b] = crc32c_tk(k, b);
    for (uint32_t j = 0; j < 6; j++) crc32c_shift_table(4ull << j, &h[kLabL5Off + 1024 * (1 + j)]);
    {
        const uint64_t zs[5] = {32, 1024, 128, 256, 512};
        for (uint32_t k = 0; k < 5; k++) crc32c_shift_table(zs[k], &h[kLabStageOff + 1024 * k]);
        const uint64_t zw[5] = {1024, 128, 256, 512, 32};
        for (uint32_t k = 0; k < 5; k++) crc32c_shift_table(zw[k], &h[kLabWinOff + 1024 * k]);
    }
    CK(hipMemcpy(d, h.data(), kLabTabBytes, hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    g_cus = prop.multiProcessorCount;
}

template <int WG, int WIN>
static void L_lane_perm(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *,
                        hipStream_t st) {
    uint32_t grid = std::min<uint32_t>((n + WG - 1) / WG, g_cus);
    hipLaunchKernelGGL((k_lane_perm<WG, WIN>), dim3(grid), dim3(WG), 0, st, s, len, h, n, o);
}
template <int CH, int NB, int WAVES, int MODE>
static void L_chunk(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    const uint32_t set = CH == 64 ? 0 : CH == 128 ? 1 : 2;
    const uint32_t tiles = (n + 63) / 64;
    uint32_t grid = std::min<uint32_t>((tiles + WAVES - 1) / WAVES, g_cus);
    hipLaunchKernelGGL((k_chunk<CH, NB, WAVES, MODE>), dim3(grid), dim3(64 * WAVES), 0, st, s, len, h, n, o,
                       tabs + set * kLabNB * 1024);
}
template <int UNR, int WPC>
static void L_stream(const uint8_t *s, uint64_t len, const bhg_handle *, uint32_t, bhg_desc *o, const uint32_t *,
                     hipStream_t st) {
    hipLaunchKernelGGL((k_stream<UNR>), dim3(g_cus * WPC), dim3(256), 0, st, s, len, o);
}

template <int G, int WAVES, int U, int MODE>
static void L_braid(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    constexpr int LG = G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3 : G == 16 ? 4 : 5;
    const uint32_t tiles = (n + 63) / 64;
    uint32_t grid = std::min<uint32_t>((tiles + WAVES - 1) / WAVES, g_cus);
    hipLaunchKernelGGL((k_braid<G, WAVES, U, MODE>), dim3(grid), dim3(64 * WAVES), 0, st, s, len, h, n, o,
                       tabs + kLabBraidOff + (LG - 1) * kLabBraidSet);
}

template <int CH, int NB, int WAVES, int MODE>
static void L_chunk2(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                     hipStream_t st) {
    const uint32_t set = CH == 64 ? 0 : CH == 128 ? 1 : 2;
    const uint32_t tiles = (n + 63) / 64;
    uint32_t grid = std::min<uint32_t>((tiles + WAVES - 1) / WAVES, g_cus);
    hipLaunchKernelGGL((k_chunk2<CH, NB, WAVES, MODE>), dim3(grid), dim3(64 * WAVES), 0, st, s, len, h, n, o,
                       tabs + set * kLabNB * 1024);
}

template <int TB, int WPC>
static void L_tiles(const uint8_t *s, uint64_t len, const bhg_handle *, uint32_t, bhg_desc *o, const uint32_t *,
                    hipStream_t st) {
    hipLaunchKernelGGL((k_tiles<TB>), dim3(g_cus * WPC), dim3(256), 0, st, s, len, o);
}
template <int RB, int WPC>
static void L_lanes(const uint8_t *s, uint64_t len, const bhg_handle *, uint32_t, bhg_desc *o, const uint32_t *,
                    hipStream_t st) {
    hipLaunchKernelGGL((k_lanes<RB>), dim3(g_cus * WPC), dim3(256), 0, st, s, len, o);
}

template <int RL, int MODE, int WPC>
static void L_lrec(const uint8_t *s, uint64_t len, const bhg_handle *, uint32_t, bhg_desc *o, const uint32_t *,
                   hipStream_t st) {
    hipLaunchKernelGGL((k_lrec<RL, MODE>), dim3(g_cus * WPC), dim3(256), 0, st, s, len, o);
}

template <int CH, int OFF, int MODE, int WPC>
static void L_cdiag(const uint8_t *s, uint64_t len, const bhg_handle *, uint32_t, bhg_desc *o, const uint32_t *,
                    hipStream_t st) {
    hipLaunchKernelGGL((k_cdiag<CH, OFF, MODE>), dim3(g_cus * WPC), dim3(256), 0, st, s, len, o);
}

template <int WG, int MODE, int WPC>
static void L_lane3(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *,
                    hipStream_t st) {
    uint32_t grid = std::min<uint32_t>((n + WG - 1) / WG, g_cus * WPC);
    hipLaunchKernelGGL((k_lane3<WG, MODE>), dim3(grid), dim3(WG), 0, st, s, len, h, n, o);
}

template <int WAVES, int PF, int WPC, int TR = 64>
static void L_gridload(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *,
                       hipStream_t st) {
    const uint32_t tiles = (n + TR - 1) / TR;
    uint32_t grid = std::min<uint32_t>((tiles + WAVES - 1) / WAVES, g_cus * WPC);
    hipLaunchKernelGGL((k_gridload<WAVES, PF, TR>), dim3(grid), dim3(64 * WAVES), 0, st, s, len, h, n, o);
}

template <int WAVES, int MODE, int RPR>
static void L_sweep(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    const uint32_t rounds = (n + RPR - 1) / RPR;
    uint32_t grid = std::min<uint32_t>((rounds + WAVES - 1) / WAVES, g_cus);
    hipLaunchKernelGGL((k_sweep<WAVES, MODE>), dim3(grid), dim3(64 * WAVES), 0, st, s, len, h, n, o,
                       tabs + kLabZ128Off, (uint32_t)RPR);
}

template <int WAVES, int RPR, int WPC = 1>
static void L_sweep2(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                     hipStream_t st) {
    const uint32_t rounds = (n + RPR - 1) / RPR;
    uint32_t grid = std::min<uint32_t>((rounds + WAVES - 1) / WAVES, g_cus * WPC);
    hipLaunchKernelGGL((k_sweep2<WAVES>), dim3(grid), dim3(64 * WAVES), 0, st, s, len, h, n, o, tabs + kLabPlainOff,
                       (uint32_t)RPR);
}

template <int NCH>
static void L_ccompute(const uint8_t *s, uint64_t len, const bhg_handle *, uint32_t, bhg_desc *o, const uint32_t *tabs,
                       hipStream_t st) {
    hipLaunchKernelGGL((k_ccompute<NCH, 0>), dim3(g_cus), dim3(1024), 0, st, s, len, o, tabs + kLabPlainOff);
}

template <int WG, int MODE, int WPC = 1>
static void L_lane5(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    uint32_t grid = std::min<uint32_t>((n + WG - 1) / WG, g_cus * WPC);
    hipLaunchKernelGGL((k_lane5<WG, MODE>), dim3(grid), dim3(WG), 0, st, s, len, h, n, o, tabs + kLabL5Off);
}

template <int R, int MODE, int WPC = 1>
static void L_stage(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    const uint32_t ng = (n + 31) / 32;
    uint32_t grid = std::min<uint32_t>(ng, g_cus * WPC);
    hipLaunchKernelGGL((k_stage<32, 8, 128, R, 34816, MODE>), dim3(grid), dim3(256), 0, st, s, len, h, n, o,
                       tabs + kLabStageOff);
}

template <int WPB, int R, int MODE, int WPC = 1>
static void L_win(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                  hipStream_t st) {
    const uint32_t ng = (n + 7) / 8;
    uint32_t grid = std::min<uint32_t>((ng + WPB - 1) / WPB, g_cus * WPC);
    hipLaunchKernelGGL((k_win<WPB, R, MODE>), dim3(grid), dim3(64 * WPB), 0, st, s, len, h, n, o, tabs + kLabWinOff);
}

template <int WPB, int R, int MODE, int WPC = 1>
static void L_tile(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                   hipStream_t st) {
    const uint32_t nt = (n + 63) / 64;
    uint32_t grid = std::min<uint32_t>((nt + WPB - 1) / WPB, g_cus * WPC);
    hipLaunchKernelGGL((k_tile<WPB, R, MODE>), dim3(grid), dim3(64 * WPB), 0, st, s, len, h, n, o, tabs + kLabWinOff);
}

template <int WPB, class Tab, int MODE, int WPC = 1>
static void L_tile2(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    const uint32_t nt = (n + 63) / 64;
    uint32_t grid = std::min<uint32_t>((nt + WPB - 1) / WPB, g_cus * WPC);
    hipLaunchKernelGGL((k_tile2<WPB, Tab, MODE>), dim3(grid), dim3(64 * WPB), 0, st, s, len, h, n, o, tabs + kLabWinOff);
}

template <int WPB, class Tab, int MODE, int PD, int WPC = 1>
static void L_tile3(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    const uint32_t nt = (n + 63) / 64;
    uint32_t grid = std::min<uint32_t>((nt + WPB - 1) / WPB, g_cus * WPC);
    hipLaunchKernelGGL((k_tile3<WPB, Tab, MODE, PD>), dim3(grid), dim3(64 * WPB), 0, st, s, len, h, n, o, tabs + kLabWinOff);
}

template <int WPB, int PD, int MODE, int WPC = 1>
static void L_tile4(const uint8_t *s, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *o, const uint32_t *tabs,
                    hipStream_t st) {
    const uint32_t nt = (n + 63) / 64;
    uint32_t grid = std::min<uint32_t>((nt + WPB - 1) / WPB, g_cus * WPC);
    hipLaunchKernelGGL((k_tile4<WPB, PD, MODE>), dim3(grid), dim3(64 * WPB), 0, st, s, len, h, n, o, tabs + kLabWinOff);
}

struct LabEntry {
    const char *name;
    launch_fn fn;
    bool diag;
};
static const LabEntry kLab[] = {
    {"tile4_w8_pd1", L_tile4<8, 1, 0>, false},
    {"tile4_w8_pd2", L_tile4<8, 2, 0>, false},
    {"tile4_w8_pd3", L_tile4<8, 3, 0>, false},
    {"tile4_w8_pd2_loads", L_tile4<8, 2, 4>, true},
    {"tile4_w8_pd3_loads", L_tile4<8, 3, 4>, true},
    {"tile4_w8_pd2_nod", L_tile4<8, 2, 16>, true},
    {"tile4_w8_pd2_compute", L_tile4<8, 2, 2>, true},
    {"tile3_w8_pd2", L_tile3<8, Crc4Perm, 0, 2>, false},
    {"tile3_w8_pd3", L_tile3<8, Crc4Perm, 0, 3>, false},
    {"tile3_w8_pd1", L_tile3<8, Crc4Perm, 0, 1>, false},
    {"tile3_w8_pd2_loads_nop1", L_tile3<8, Crc4Perm, 4 | 8, 2>, true},
    {"tile3_w8_pd3_loads_nop1", L_tile3<8, Crc4Perm, 4 | 8, 3>, true},
    {"tile3_w8_pd2_loads_nop1_nod", L_tile3<8, Crc4Perm, 4 | 8 | 16, 2>, true},
    {"tile3_w8_pd1_loads_nop1_nod", L_tile3<8, Crc4Perm, 4 | 8 | 16, 1>, true},
    {"tile3_w8_pd2_nod", L_tile3<8, Crc4Perm, 16, 2>, true},
    {"tile2_perm_w8_compute", L_tile2<8, Crc4Perm, 2, 1>, true},
    {"tile2_perm_w8_loads", L_tile2<8, Crc4Perm, 4, 1>, true},
    {"tile2_perm_w16_sb_compute", L_tile2<16, Crc4Perm, 3, 1>, true},
    {"tile2_perm_w16_sb_loads", L_tile2<16, Crc4Perm, 5, 1>, true},
    {"tile2_perm_w8_loads_nop1", L_tile2<8, Crc4Perm, 4 | 8, 1>, true},
    {"tile2_perm_w8_nop1", L_tile2<8, Crc4Perm, 8, 1>, true},
    {"tile2_perm_w16_sb_loads_nop1", L_tile2<16, Crc4Perm, 5 | 8, 1>, true},
    {"tile2_perm_w16", L_tile2<16, Crc4Perm, 0, 1>, false},
    {"tile2_perm_w16_sb", L_tile2<16, Crc4Perm, 1, 1>, false},
    {"tile2_perm_w8", L_tile2<8, Crc4Perm, 0, 1>, false},
    {"tile2_perm_w12_sb", L_tile2<12, Crc4Perm, 1, 1>, false},
    {"tile2_r16_w8_sb", L_tile2<8, Crc4Lds<16>, 1, 2>, false},
    {"tile_w4_r4_x4", L_tile<4, 4, 0, 4>, false},
    {"tile_w4_r8_x3", L_tile<4, 8, 0, 3>, false},
    {"tile_w8_r8_x2", L_tile<8, 8, 0, 2>, false},
    {"tile_w8_r16_x2", L_tile<8, 16, 0, 2>, false},
    {"tile_w16_r16_x1", L_tile<16, 16, 0, 1>, false},
    {"tile_w4_r4_x8", L_tile<4, 4, 0, 8>, false},
    {"win_w4_r4_x4", L_win<4, 4, 0, 4>, false},
    {"win_w4_r8_x3", L_win<4, 8, 0, 3>, false},
    {"win_w8_r16_x2", L_win<8, 16, 0, 2>, false},
    {"win_w8_r8_x2", L_win<8, 8, 0, 2>, false},
    {"win_w4_r4_x8", L_win<4, 4, 0, 8>, false},
    {"win_w16_r16_x1", L_win<16, 16, 0, 1>, false},
    {"stage_r8", L_stage<8, 0>, false},
    {"stage_r16", L_stage<16, 0>, false},
    {"stage_r8_nofb", L_stage<8, 1>, false},
    {"stream_u4_w8", L_stream<4, 8>, true},
    {"stream_u8_w8", L_stream<8, 8>, true},
    {"stream_u4_w16", L_stream<4, 16>, true},
    {"lane5_wg1024", L_lane5<1024, 0>, false},
    {"lane5_wg512", L_lane5<512, 0>, false},
    {"lane5_wg1024_loads", L_lane5<1024, 1>, true},
    {"lane5_wg512_loads", L_lane5<512, 1>, true},
    {"lane5_wg512_loads_np", L_lane5<512, 1 | 4>, true},
    {"lane5_wg512_loads_nd", L_lane5<512, 1 | 8>, true},
    {"lane5_wg512_loads_np_nd", L_lane5<512, 1 | 4 | 8>, true},
    {"lane5_wg512_np_nd", L_lane5<512, 4 | 8>, true},
    {"lane5_wg1024_np", L_lane5<1024, 4>, true},
    {"ccompute_1", L_ccompute<1>, true},
    {"ccompute_2", L_ccompute<2>, true},
    {"ccompute_4", L_ccompute<4>, true},
    {"sweep2_w16_r7", L_sweep2<16, 7>, false},
    {"sweep2_w8_r7", L_sweep2<8, 7>, false},
    {"sweep2_w16_r14", L_sweep2<16, 14>, false},
    {"sweep2_w8_r14", L_sweep2<8, 14>, false},
    {"sweep_w16_r7", L_sweep<16, 0, 7>, false},
    {"sweep_w8_r7", L_sweep<8, 0, 7>, false},
    {"sweep_w16_r6", L_sweep<16, 0, 6>, false},
    {"sweep_w16_r14", L_sweep<16, 0, 14>, false},
    {"sweep_w16_r7_loads", L_sweep<16, 1, 7>, true},
    {"gridload_w4_pf0_x4_tr8", L_gridload<4, 0, 4, 8>, true},
    {"gridload_w4_pf0_x4_tr16", L_gridload<4, 0, 4, 16>, true},
    {"gridload_w4_pf0_x4_tr32", L_gridload<4, 0, 4, 32>, true},
    {"gridload_w4_pf0_x1", L_gridload<4, 0, 1>, true},
    {"gridload_w4_pf0_x2", L_gridload<4, 0, 2>, true},
    {"gridload_w8_pf0_x1", L_gridload<8, 0, 1>, true},
    {"gridload_w16_pf0", L_gridload<16, 0, 1>, true},
    {"gridload_w4_pf0_x8", L_gridload<4, 0, 8>, true},
    {"gridload_w16_pf1", L_gridload<16, 1, 1>, true},
    {"gridload_w8_pf1", L_gridload<8, 1, 1>, true},
    {"gridload_w4_pf1_x4", L_gridload<4, 1, 4>, true},
    {"gridload_w4_pf0_x4", L_gridload<4, 0, 4>, true},
    {"lane3_wg512", L_lane3<512, 0, 1>, false},
    {"lane3_wg1024", L_lane3<1024, 0, 1>, false},
    {"lane3_wg256", L_lane3<256, 0, 1>, false},
    {"lane3_wg512_loads", L_lane3<512, 1, 1>, true},
    {"lane3_wg1024_loads", L_lane3<1024, 1, 1>, true},
    {"lane_perm_wg1024_win8", L_lane_perm<1024, 8>, false},
    {"lane_perm_wg512_win8", L_lane_perm<512, 8>, false},
    {"lane_perm_wg1024_win4", L_lane_perm<1024, 4>, false},
    {"stream_u4_w4", L_stream<4, 4>, true},
    {"tiles_1k_w8", L_tiles<1024, 8>, true},
    {"tiles_4k_w4", L_tiles<4096, 4>, true},
    {"tiles_8k_w4", L_tiles<8192, 4>, true},
    {"tiles_8k_w2", L_tiles<8192, 2>, true},
    {"tiles_64k_w4", L_tiles<65536, 4>, true},
    {"tiles_64k_w1", L_tiles<65536, 1>, true},
    {"lrec_1076_al128_w4", L_lrec<1076, 2, 4>, true},
    {"lrec_1040_al16_w4", L_lrec<1040, 1, 4>, true},
    {"lrec_1088_al16_w4", L_lrec<1088, 1, 4>, true},
    {"lrec_1152_al16_w4", L_lrec<1152, 1, 4>, true},
    {"lrec_1280_al16_w4", L_lrec<1280, 1, 4>, true},
    {"lrec_2048_al16_w4", L_lrec<2048, 1, 4>, true},
    {"lrec_1536_al16_w4", L_lrec<1536, 1, 4>, true},
    {"lrec_512_al16_w4", L_lrec<512, 1, 4>, true},
    {"lrec_1076_unal_w4", L_lrec<1076, 0, 4>, true},
    {"lrec_1076_al16_w4", L_lrec<1076, 1, 4>, true},
    {"lrec_1024_unal_w4", L_lrec<1024, 0, 4>, true},
    {"lrec_1028_unal_w4", L_lrec<1028, 0, 4>, true},
    {"lrec_1028_al16_w4", L_lrec<1028, 1, 4>, true},
    {"lrec_1076_al16_w2", L_lrec<1076, 1, 2>, true},
    {"lrec_1076_al16_w8", L_lrec<1076, 1, 8>, true},
    {"lanes_64_w4", L_lanes<64, 4>, true},
    {"lanes_128_w4", L_lanes<128, 4>, true},
    {"lanes_1k_w4", L_lanes<1024, 4>, true},
    {"lanes_1k_w2", L_lanes<1024, 2>, true},
    {"stream_u2_w4", L_stream<2, 4>, true},
    {"stream_u1_w8", L_stream<1, 8>, true},
    {"chunk2_128_w16", L_chunk2<128, 5, 16, 0>, false},
    {"chunk2_64_w16", L_chunk2<64, 5, 16, 0>, false},
    {"chunk2_128_w8", L_chunk2<128, 5, 8, 0>, false},
    {"chunk2_128_w12", L_chunk2<128, 5, 12, 0>, false},
    {"chunk2_128_loads", L_chunk2<128, 5, 16, 1>, true},
    {"chunk2_64_loads", L_chunk2<64, 5, 16, 1>, true},
    {"chunk64_nb5_w16", L_chunk<64, 5, 16, 0>, false},
    {"chunk128_nb5_w16", L_chunk<128, 5, 16, 0>, false},
    {"chunk256_nb4_w16", L_chunk<256, 4, 16, 0>, false},
    {"chunk128_nb5_w8", L_chunk<128, 5, 8, 0>, false},
    {"chunk128_loadsonly", L_chunk<128, 5, 16, 1>, true},
    {"chunk128_loads_noparse", L_chunk<128, 5, 16, 1 | 4>, true},
    {"chunk128_loads_noparse_nodesc", L_chunk<128, 5, 16, 1 | 4 | 8>, true},
    {"chunk128_noparse", L_chunk<128, 5, 16, 4>, true},
    {"cdiag128_off52_unal", L_cdiag<128, 52, 0, 4>, true},
    {"cdiag128_off52_al16", L_cdiag<128, 52, 1, 4>, true},
    {"cdiag128_off48_al16", L_cdiag<128, 48, 1, 4>, true},
    {"cdiag128_off0", L_cdiag<128, 0, 1, 4>, true},
    {"cdiag64_off52_unal", L_cdiag<64, 52, 0, 4>, true},
    {"chunk128_computeonly", L_chunk<128, 5, 16, 2>, true},
};
static const int kNumLab = sizeof(kLab) / sizeof(kLab[0]);
