// rf_tfr.hip — tf.train.Example records -> batched CSR on the GPU (include/rf_io.h "device parse").
//
// The same columns Reader::parse (rf_io.cpp) produces on the host — parse_example's output for
// FixedLen[Sequence]Feature descriptions (backend/core/dataloader.py:23-44, 77-89) — computed from
// the serialized records after they are streamed to HBM, so the host only frames, CRC-checks and
// packs records (rf_tfr_next_records). Four stream-ordered steps:
//
//   count   one wave per record. The record is staged in LDS (coalesced 16-byte loads; records
//           longer than the slot are parsed from HBM). Lane 0 walks the Example / Features framing
//           and hands map entries out 64 at a time; every lane parses one entry (key, Feature),
//           looks the key up in the schema hash (rf_tfr_blob.h) and keeps the LAST entry of each key
//           (LDS atomic max of the entry position — later entries sit later in the record). Then
//           lanes stride over the schema: re-read the winning entry, type-check it and count its
//           values (value count, token bytes) exactly as count_list does; lmax by atomic max, the
//           first error of the record (schema order) by a wave min, the first failing record by
//           an atomic min.
//   scan    exclusive prefix sums of the per-(example, slot) counts in example-major order: the
//           CSR offsets bag_off / ibag_off / fbag_off and the token byte starts (3 launches: tile
//           sums, one block per array over tile sums, apply). The totals land in the stats.
//   write   one wave per record again: lanes stride over the schema and write token offsets and
//           bytes, int64 / float values and scalars (defaults where a key is missing). Nothing is
//           written when the batch has an error.
//
// All work is integer/byte movement; the bound is the sequential protobuf walk per record (LDS
// latency), spread over thousands of records in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "../../include/rf_api.h"
#include "../../include/rf_io.h"
#include "rf_tfr_blob.h"

static_assert(sizeof(rf_tfr_dev_stats) == 64, "rf_tfr_dev_stats layout");

int rf_set_error(int code, const char* fmt, ...);  // rf_api.cpp

namespace {

constexpr int kEnt = 64;          // map entries handed from the walker lane per round
constexpr int kLdsBudget = 65536; // per workgroup (one wave)
constexpr int kMaxFeatures = 8192;
constexpr int kTile = 2048;       // scan tile (256 threads x 8)
constexpr int kScanArrays = 4;    // tok count, tok bytes, int64 count, float count

struct Schema {
    const TfrBlobHdr* h;
    const TfrBlobFeat* f;
    const int32_t* ht;
    const uint8_t* names;
};

__device__ __forceinline__ Schema schema_of(const uint8_t* blob) {
    Schema s;
    s.h = reinterpret_cast<const TfrBlobHdr*>(blob);
    s.f = reinterpret_cast<const TfrBlobFeat*>(blob + sizeof(TfrBlobHdr));
    s.ht = reinterpret_cast<const int32_t*>(blob + sizeof(TfrBlobHdr) + sizeof(TfrBlobFeat) * s.h->F);
    s.names = blob + s.h->names_off;
    return s;
}

// ---- protobuf wire format (the rules of rf_io.cpp's get_varint / skip_field / get_span) ----------
__device__ __forceinline__ bool d_varint(const uint8_t*& p, const uint8_t* e, uint64_t* v) {
    uint64_t r = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
        const uint32_t b = *p++;
        r |= static_cast<uint64_t>(b & 0x7f) << s;
        if (!(b & 0x80)) {
            *v = r;
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ bool d_skip(const uint8_t*& p, const uint8_t* e, uint32_t wt) {
    uint64_t v;
    switch (wt) {
        case 0: return d_varint(p, e, &v);
        case 1: if (e - p < 8) return false; p += 8; return true;
        case 2: if (!d_varint(p, e, &v) || static_cast<uint64_t>(e - p) < v) return false; p += v; return true;
        case 5: if (e - p < 4) return false; p += 4; return true;
        default: return false;
    }
}

__device__ __forceinline__ bool d_span(const uint8_t*& p, const uint8_t* e, const uint8_t** s, uint32_t* n) {
    uint64_t v;
    if (!d_varint(p, e, &v) || static_cast<uint64_t>(e - p) < v) return false;
    *s = p;
    *n = static_cast<uint32_t>(v);
    p += v;
    return true;
}

// Map entry {1: key, 2: Feature} at payload [p, p + n).
__device__ __forceinline__ bool d_map_entry(const uint8_t* p, uint32_t n, const uint8_t** key, uint32_t* key_n,
                                            const uint8_t** val, uint32_t* val_n, bool* has_val) {
    const uint8_t* e = p + n;
    *key = nullptr;
    *key_n = 0;
    *has_val = false;
    while (p < e) {
        uint64_t t;
        if (!d_varint(p, e, &t)) return false;
        if (t == ((1u << 3) | 2)) {
            if (!d_span(p, e, key, key_n)) return false;
        } else if (t == ((2u << 3) | 2)) {
            if (!d_span(p, e, val, val_n)) return false;
            *has_val = true;
        } else if (!d_skip(p, e, static_cast<uint32_t>(t & 7))) {
            return false;
        }
    }
    return true;
}

// Feature -> (kind, list span); kind -2 = no kind field. The last kind field wins (oneof).
__device__ __forceinline__ bool d_feature(const uint8_t* p, uint32_t n, int* kind, const uint8_t** lp, uint32_t* ln) {
    const uint8_t* e = p + n;
    *kind = -2;
    *lp = nullptr;
    *ln = 0;
    while (p < e) {
        uint64_t t;
        if (!d_varint(p, e, &t)) return false;
        const uint32_t field = static_cast<uint32_t>(t >> 3), wt = static_cast<uint32_t>(t & 7);
        if (wt == 2 && field >= 1 && field <= 3) {
            if (!d_span(p, e, lp, ln)) return false;
            *kind = field == 1 ? RF_TFR_BYTES : field == 2 ? RF_TFR_FLOAT : RF_TFR_INT64;
        } else if (!d_skip(p, e, wt)) {
            return false;
        }
    }
    return true;
}

// Values (and BytesList payload bytes) of a list; false if malformed (rf_io.cpp count_list).
__device__ __forceinline__ bool d_count_list(const uint8_t* p, uint32_t n, int kind, int32_t* count, int32_t* nbytes) {
    const uint8_t* e = p + n;
    int32_t c = 0, b = 0;
    while (p < e) {
        uint64_t t;
        if (!d_varint(p, e, &t)) return false;
        const uint32_t field = static_cast<uint32_t>(t >> 3), wt = static_cast<uint32_t>(t & 7);
        if (field != 1) {
            if (!d_skip(p, e, wt)) return false;
            continue;
        }
        if (kind == RF_TFR_BYTES) {
            const uint8_t* v;
            uint32_t vn;
            if (wt != 2 || !d_span(p, e, &v, &vn)) return false;
            ++c;
            b += static_cast<int32_t>(vn);
        } else if (kind == RF_TFR_FLOAT) {
            if (wt == 5) {
                if (e - p < 4) return false;
                p += 4;
                ++c;
            } else if (wt == 2) {
                const uint8_t* v;
                uint32_t vn;
                if (!d_span(p, e, &v, &vn) || (vn & 3)) return false;
                c += static_cast<int32_t>(vn / 4);
            } else {
                return false;
            }
        } else {
            if (wt == 0) {
                uint64_t x;
                if (!d_varint(p, e, &x)) return false;
                ++c;
            } else if (wt == 2) {
                const uint8_t* v;
                uint32_t vn;
                if (!d_span(p, e, &v, &vn)) return false;
                const uint8_t* qe = v + vn;
                while (v < qe) {
                    uint64_t x;
                    if (!d_varint(v, qe, &x)) return false;
                    ++c;
                }
            } else {
                return false;
            }
        }
    }
    *count = c;
    *nbytes = b;
    return true;
}

__device__ __forceinline__ int d_lookup(const Schema& S, const uint8_t* key, uint32_t n) {
    uint32_t h = 2166136261u;
    for (uint32_t i = 0; i < n; ++i) h = (h ^ key[i]) * 16777619u;
    const uint32_t m = static_cast<uint32_t>(S.h->hmask);
    for (uint32_t s = h & m;; s = (s + 1) & m) {
        const int j = S.ht[s];
        if (j < 0) return -1;
        const TfrBlobFeat& f = S.f[j];
        if (static_cast<uint32_t>(f.name_len) == n) {
            const uint8_t* nm = S.names + f.name_off;
            uint32_t i = 0;
            while (i < n && nm[i] == key[i]) ++i;
            if (i == n) return j;
        }
    }
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}

// Copies record bytes [r0, r0 + n) into LDS at slot + (r0 & 15) with 16-byte loads (the packed
// buffer is readable 16 bytes past the last record, rf_io.h).
__device__ __forceinline__ void stage(uint8_t* slot, const uint8_t* rec, int64_t r0, uint32_t n, int lane) {
    const int64_t a0 = r0 & ~int64_t{15};
    const int nw = static_cast<int>(((r0 - a0) + n + 15) >> 4);
    const uint4* src = reinterpret_cast<const uint4*>(rec + a0);
    uint4* dst = reinterpret_cast<uint4*>(slot);
    for (int i = lane; i < nw; i += 256) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = src[min(i + 64 * k, nw - 1)];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + 64 * k < nw) dst[i + 64 * k] = v[k];
    }
}

// Error word of one (record, key): ordered by schema index, then by the check order of Reader::parse.
struct Err {
    int type, feat, kind, count;
};

struct CountArgs {
    const uint8_t* blob;
    const uint8_t* rec;
    const int64_t* rec_off;
    int32_t B, slot_bytes;
    int4* spans;  // [B*F] {list offset in record, list bytes, kind (-1 absent), value count}
    int32_t *tokc, *tokb, *ic, *fc;
    int32_t *lmax, *ilmax, *flmax;
    int4* err_rec;  // [B] {type, feat, kind, count}
    rf_tfr_dev_stats* stats;
};

__device__ __forceinline__ void lmax_update(int32_t* p, int32_t v) {
    if (v > __builtin_nontemporal_load(p)) atomicMax(p, v);
}

// Pass over one record at r[0, n) (r is LDS when staged: the compiler sees that address space in
// that instantiation).
__device__ __forceinline__ void count_record(const CountArgs& a, const Schema& S, const uint8_t* r, uint32_t n, int b,
                                             int32_t* win, uint32_t* ent, int lane) {
    const int F = S.h->F;
    for (int j = lane; j < F; j += 64) win[j] = -1;
    uint32_t p = 0, fp = 0, fe = 0;  // walker (lane 0): Example cursor, current Features span
    int bad = 0;
    __syncthreads();
    for (;;) {
        int cnt = 0, wbad = 0, wdone = 0;
        if (lane == 0) {
            const uint8_t* e = r + n;
            while (cnt < kEnt) {
                if (fp < fe) {
                    const uint8_t* q = r + fp;
                    const uint8_t* qe = r + fe;
                    uint64_t tag;
                    if (!d_varint(q, qe, &tag)) { wbad = 1; break; }
                    if (tag == ((1u << 3) | 2)) {
                        const uint8_t* s;
                        uint32_t sn;
                        if (!d_span(q, qe, &s, &sn)) { wbad = 1; break; }
                        ent[cnt] = fp;  // entry position (its tag): later entries have larger ones
                        ent[kEnt + cnt] = static_cast<uint32_t>(s - r);
                        ent[2 * kEnt + cnt] = sn;
                        ++cnt;
                    } else if (!d_skip(q, qe, static_cast<uint32_t>(tag & 7))) {
                        wbad = 1;
                        break;
                    }
                    fp = static_cast<uint32_t>(q - r);
                } else if (p < n) {
                    const uint8_t* q = r + p;
                    uint64_t tag;
                    if (!d_varint(q, e, &tag)) { wbad = 1; break; }
                    if (tag == ((1u << 3) | 2)) {
                        const uint8_t* s;
                        uint32_t sn;
                        if (!d_span(q, e, &s, &sn)) { wbad = 1; break; }
                        fp = static_cast<uint32_t>(s - r);
                        fe = fp + sn;
                    } else if (!d_skip(q, e, static_cast<uint32_t>(tag & 7))) {
                        wbad = 1;
                        break;
                    }
                    p = static_cast<uint32_t>(q - r);
                } else {
                    wdone = 1;
                    break;
                }
            }
        }
        cnt = __shfl(cnt, 0);
        wbad = __shfl(wbad, 0);
        wdone = __shfl(wdone, 0);
        __syncthreads();
        if (lane < cnt) {
            const uint32_t hp = ent[lane];
            const uint8_t* es = r + ent[kEnt + lane];  // the entry's payload, framed by the walker
            const uint8_t *key, *val = nullptr;
            uint32_t key_n, val_n = 0;
            bool has_val;
            if (!d_map_entry(es, ent[2 * kEnt + lane], &key, &key_n, &val, &val_n, &has_val)) {
                bad = 1;
            } else {
                const int j = d_lookup(S, key, key_n);
                if (j >= 0) {
                    int kind;
                    const uint8_t* lp;
                    uint32_t ln;
                    if (has_val && !d_feature(val, val_n, &kind, &lp, &ln)) bad = 1;
                    atomicMax(&win[j], static_cast<int32_t>(hp));
                }
            }
        }
        __syncthreads();
        if (wbad || wdone) {
            bad |= wbad;
            break;
        }
    }
    bad = wave_or(bad);

    int32_t* lm[3] = {a.lmax, a.ilmax, a.flmax};
    const int Sb = S.h->Sb, Si = S.h->Si, Sf = S.h->Sf;
    int first = INT_MAX;  // (feat << 3) | type of this lane's first error
    Err er{0, 0, 0, 0};
    for (int j = lane; j < F; j += 64) {
        int ekind = 0;
        const TfrBlobFeat f = S.f[j];
        const int w = win[j];
        int kind = -1, err = 0;
        uint32_t lo = 0, ln = 0;
        int32_t c = 0, nb = 0;
        if (!bad && w >= 0) {
            const uint8_t* h = r + w;
            uint64_t tag;
            const uint8_t *es, *key, *val = nullptr, *lp = nullptr;
            uint32_t en, key_n, val_n = 0;
            bool has_val;
            d_varint(h, r + n, &tag);
            d_span(h, r + n, &es, &en);
            d_map_entry(es, en, &key, &key_n, &val, &val_n, &has_val);
            kind = -2;
            if (has_val) d_feature(val, val_n, &kind, &lp, &ln);
            if (kind >= 0) {
                lo = static_cast<uint32_t>(lp - r);
                if (kind != f.kind) {
                    err = 2;
                    ekind = kind;
                } else if (!d_count_list(lp, ln, kind, &c, &nb)) {
                    err = 3;
                }
            } else {  // a Feature with no kind: an empty list of the schema's kind
                kind = f.kind;
                ln = 0;
            }
        }
        if (!bad && !err && f.shape == RF_TFR_SCALAR) {
            if (kind == -1) {
                c = f.kind == RF_TFR_BYTES ? 1 : 0;  // missing -> default ("" is one empty token)
            } else if (c != 1) {
                err = 4;
            }
        }
        if (err) {
            if (first == INT_MAX) {
                first = (j << 3) | err;
                er.kind = ekind;
                er.count = c;
            }
            kind = -1;
            c = nb = 0;
            ln = 0;
        }
        if (bad) c = nb = 0, kind = -1;
        const int64_t bj = static_cast<int64_t>(b) * F + j;
        a.spans[bj] = make_int4(static_cast<int>(lo), static_cast<int>(ln), kind, c);
        if (f.kind == RF_TFR_BYTES) {
            a.tokc[static_cast<int64_t>(b) * Sb + f.gpos] = c;
            a.tokb[static_cast<int64_t>(b) * Sb + f.gpos] = nb;
            if (c) lmax_update(lm[0] + f.gpos, c);
        } else if (f.shape == RF_TFR_SEQ) {
            if (f.kind == RF_TFR_INT64) {
                a.ic[static_cast<int64_t>(b) * Si + f.gpos] = c;
                if (c) lmax_update(lm[1] + f.gpos, c);
            } else {
                a.fc[static_cast<int64_t>(b) * Sf + f.gpos] = c;
                if (c) lmax_update(lm[2] + f.gpos, c);
            }
        }
    }
    const int wfirst = wave_min(bad ? 1 : first);  // a malformed Example is reported before any key
    if (wfirst != INT_MAX) {
        if (first == wfirst && !bad) {  // the lane that owns the first error writes its details
            a.err_rec[b] = make_int4(first & 7, first >> 3, er.kind, er.count);
        } else if (bad && lane == 0) {
            a.err_rec[b] = make_int4(1, 0, 0, 0);
        }
        if (lane == 0) atomicMin(&a.stats->err_b, b);
    }
}

__global__ __launch_bounds__(64) void tfr_count_kernel(CountArgs a) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const Schema S = schema_of(a.blob);
    uint8_t* slot = smem;
    int32_t* win = reinterpret_cast<int32_t*>(smem + a.slot_bytes);
    uint32_t* ent = reinterpret_cast<uint32_t*>(win + ((S.h->F + 3) & ~3));
    const int64_t r0 = a.rec_off[b];
    const uint32_t n = static_cast<uint32_t>(a.rec_off[b + 1] - r0);
    if (((r0 & 15) + n + 15) / 16 * 16 <= static_cast<uint64_t>(a.slot_bytes)) {
        stage(slot, a.rec, r0, n, lane);
        count_record(a, S, slot + (r0 & 15), n, b, win, ent, lane);
    } else {
        count_record(a, S, a.rec + r0, n, b, win, ent, lane);
    }
}

// ---- scan ----------------------------------------------------------------------------------------
struct ScanArgs {
    const int32_t* in[kScanArrays];
    int32_t* out[kScanArrays];  // N + 1 entries (exclusive prefix, total last)
    int64_t n[kScanArrays];
    int32_t* tsum;  // [kScanArrays][max_tiles]
    int32_t max_tiles;
    rf_tfr_dev_stats* stats;
    const int4* err_rec;
};

__device__ __forceinline__ int block_excl_scan256(int v, int* total) {
    __shared__ int wsum[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        pre += k < w ? wsum[k] : 0;
        tot += wsum[k];
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

__global__ __launch_bounds__(256) void tfr_scan_reduce(ScanArgs a) {
    const int k = blockIdx.y;
    const int64_t n = a.n[k];
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kTile;
    if (t0 >= n) return;
    int s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int64_t idx = t0 + threadIdx.x + 256 * i;
        if (idx < n) s += a.in[k][idx];
    }
    int tot;
    block_excl_scan256(s, &tot);
    if (threadIdx.x == 0) a.tsum[static_cast<int64_t>(k) * a.max_tiles + blockIdx.x] = tot;
}

// One block per array: tile sums -> exclusive tile prefixes (in place), totals to out[n] and the stats.
__global__ __launch_bounds__(256) void tfr_scan_tiles(ScanArgs a) {
    const int k = blockIdx.x;
    const int64_t n = a.n[k];
    const int tiles = static_cast<int>((n + kTile - 1) / kTile);
    int32_t* ts = a.tsum + static_cast<int64_t>(k) * a.max_tiles;
    int carry = 0;
    for (int t0 = 0; t0 < tiles; t0 += 256) {
        const int t = t0 + threadIdx.x;
        const int v = t < tiles ? ts[t] : 0;
        int tot;
        const int ex = block_excl_scan256(v, &tot);
        if (t < tiles) ts[t] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        if (a.out[k]) a.out[k][n] = carry;
        int64_t* tot = k == 0 ? &a.stats->n_tok : k == 1 ? &a.stats->n_tok_bytes : k == 2 ? &a.stats->n_ival : &a.stats->n_fval;
        *tot = carry;
        if (k == 0) {
            const int eb = a.stats->err_b;
            if (eb != INT_MAX) {
                const int4 e = a.err_rec[eb];
                a.stats->err_type = e.x;
                a.stats->err_feat = e.y;
                a.stats->err_kind = e.z;
                a.stats->err_count = e.w;
            }
        }
    }
}

__global__ __launch_bounds__(256) void tfr_scan_apply(ScanArgs a) {
    const int k = blockIdx.y;
    const int64_t n = a.n[k];
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kTile;
    if (t0 >= n || !a.out[k]) return;
    const int64_t base = t0 + threadIdx.x * 8;  // 8 consecutive elements per thread
    int v[8], s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = base + i < n ? a.in[k][base + i] : 0;
        s += v[i];
    }
    int tot;
    int pre = block_excl_scan256(s, &tot) + a.tsum[static_cast<int64_t>(k) * a.max_tiles + blockIdx.x];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (base + i < n) a.out[k][base + i] = pre;
        pre += v[i];
    }
}

// ---- write -----------------------------------------------------------------------------------------
struct WriteArgs {
    const uint8_t* blob;
    const uint8_t* rec;
    const int64_t* rec_off;
    int32_t B, slot_bytes;
    const int4* spans;
    const int32_t* bstart;  // token byte start per (example, bytes slot)
    rf_tfr_columns c;
    const rf_tfr_dev_stats* stats;
};

__device__ __forceinline__ void write_record(const WriteArgs& a, const Schema& S, const uint8_t* r, int b, int lane) {
    const int F = S.h->F, Sb = S.h->Sb, Si = S.h->Si, Sf = S.h->Sf, Ni = S.h->Ni, Nf = S.h->Nf;
    for (int j = lane; j < F; j += 64) {
        const TfrBlobFeat f = S.f[j];
        const int4 sp = a.spans[static_cast<int64_t>(b) * F + j];
        const uint8_t* p = r + sp.x;
        const uint8_t* e = p + sp.y;
        const bool present = sp.z >= 0;
        if (f.kind == RF_TFR_BYTES) {
            const int64_t bg = static_cast<int64_t>(b) * Sb + f.gpos;
            int32_t t = a.c.bag_off[bg];
            int32_t cur = a.bstart[bg];
            if (present) {
                while (p < e) {
                    uint64_t tag = 0;
                    d_varint(p, e, &tag);
                    if ((tag >> 3) != 1) {
                        d_skip(p, e, static_cast<uint32_t>(tag & 7));
                        continue;
                    }
                    const uint8_t* v;
                    uint32_t vn;
                    d_span(p, e, &v, &vn);
                    a.c.tok_off[t++] = cur;
                    uint8_t* dst = a.c.tok_bytes + cur;
                    for (uint32_t i = 0; i < vn; ++i) dst[i] = v[i];
                    cur += static_cast<int32_t>(vn);
                }
            } else if (sp.w == 1) {  // missing SCALAR bytes -> b""
                a.c.tok_off[t] = cur;
            }
        } else if (f.kind == RF_TFR_INT64) {
            int64_t one = f.def_i;
            const bool seq = f.shape == RF_TFR_SEQ;
            int64_t* dst = seq ? a.c.ival + a.c.ibag_off[static_cast<int64_t>(b) * Si + f.gpos] : nullptr;
            if (present) {
                while (p < e) {
                    uint64_t tag = 0, x = 0;
                    d_varint(p, e, &tag);
                    if ((tag >> 3) != 1) {
                        d_skip(p, e, static_cast<uint32_t>(tag & 7));
                        continue;
                    }
                    if ((tag & 7) == 0) {
                        d_varint(p, e, &x);
                        if (seq) *dst++ = static_cast<int64_t>(x);
                        else one = static_cast<int64_t>(x);
                    } else {
                        const uint8_t* v;
                        uint32_t vn;
                        d_span(p, e, &v, &vn);
                        const uint8_t* qe = v + vn;
                        while (v < qe) {
                            d_varint(v, qe, &x);
                            if (seq) *dst++ = static_cast<int64_t>(x);
                            else one = static_cast<int64_t>(x);
                        }
                    }
                }
            }
            if (!seq) a.c.iscalar[static_cast<int64_t>(b) * Ni + f.gpos] = one;
        } else {
            float one = f.def_f;
            const bool seq = f.shape == RF_TFR_SEQ;
            float* dst = seq ? a.c.fval + a.c.fbag_off[static_cast<int64_t>(b) * Sf + f.gpos] : nullptr;
            if (present) {
                while (p < e) {
                    uint64_t tag = 0;
                    d_varint(p, e, &tag);
                    if ((tag >> 3) != 1) {
                        d_skip(p, e, static_cast<uint32_t>(tag & 7));
                        continue;
                    }
                    const uint8_t* v = p;
                    uint32_t vn = 4;
                    if ((tag & 7) == 5) {
                        p += 4;
                    } else {
                        d_span(p, e, &v, &vn);
                    }
                    for (uint32_t i = 0; i < vn; i += 4) {
                        const uint32_t u = static_cast<uint32_t>(v[i]) | (static_cast<uint32_t>(v[i + 1]) << 8) |
                                           (static_cast<uint32_t>(v[i + 2]) << 16) | (static_cast<uint32_t>(v[i + 3]) << 24);
                        if (seq) *dst++ = __uint_as_float(u);
                        else one = __uint_as_float(u);
                    }
                }
            }
            if (!seq) a.c.fscalar[static_cast<int64_t>(b) * Nf + f.gpos] = one;
        }
    }
}

__global__ __launch_bounds__(64) void tfr_write_kernel(WriteArgs a) {
    extern __shared__ __align__(16) uint8_t smem[];
    if (a.stats->err_b != INT_MAX) return;  // the batch fails as a whole: write nothing
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const Schema S = schema_of(a.blob);
    if (b == 0 && lane == 0 && S.h->Sb) {
        const int64_t nt = a.stats->n_tok;
        a.c.tok_off[nt] = static_cast<int32_t>(a.stats->n_tok_bytes);
    }
    const int64_t r0 = a.rec_off[b];
    const uint32_t n = static_cast<uint32_t>(a.rec_off[b + 1] - r0);
    if (((r0 & 15) + n + 15) / 16 * 16 <= static_cast<uint64_t>(a.slot_bytes)) {
        stage(smem, a.rec, r0, n, lane);
        __syncthreads();
        write_record(a, S, smem + (r0 & 15), b, lane);
    } else {
        write_record(a, S, a.rec + r0, b, lane);
    }
}

__global__ void tfr_init_kernel(rf_tfr_dev_stats* st, int32_t* lmax, int Sb, int32_t* ilmax, int Si, int32_t* flmax, int Sf) {
    const int i = threadIdx.x + blockIdx.x * blockDim.x;
    if (i == 0) {
        st->n_tok_bytes = st->n_tok = st->n_ival = st->n_fval = 0;
        st->err_b = INT_MAX;
        st->err_type = st->err_feat = st->err_kind = 0;
        st->err_count = 0;
        st->reserved = 0;
    }
    if (i < Sb) lmax[i] = 0;
    if (i < Si) ilmax[i] = 0;
    if (i < Sf) flmax[i] = 0;
}

struct Workspace {
    int4* spans;
    int32_t *tokc, *tokb, *bstart, *ic, *fc, *tsum;
    int4* err_rec;
    int32_t max_tiles;
    int64_t bytes;
};

inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t{255}; }

Workspace plan(const TfrBlobHdr& h, int64_t B, uint8_t* base) {
    Workspace w{};
    const int64_t nmax = B * std::max(std::max(h.Sb, h.Si), std::max(h.Sf, 1));
    w.max_tiles = static_cast<int32_t>((nmax + kTile - 1) / kTile);
    int64_t o = 0;
    auto take = [&](int64_t bytes) {
        uint8_t* p = base ? base + o : nullptr;
        o += align256(bytes);
        return p;
    };
    w.spans = reinterpret_cast<int4*>(take(16 * B * h.F));
    w.tokc = reinterpret_cast<int32_t*>(take(4 * B * h.Sb));
    w.tokb = reinterpret_cast<int32_t*>(take(4 * B * h.Sb));
    w.bstart = reinterpret_cast<int32_t*>(take(4 * (B * h.Sb + 1)));
    w.ic = reinterpret_cast<int32_t*>(take(4 * B * h.Si));
    w.fc = reinterpret_cast<int32_t*>(take(4 * B * h.Sf));
    w.err_rec = reinterpret_cast<int4*>(take(16 * B));
    w.tsum = reinterpret_cast<int32_t*>(take(4 * int64_t{kScanArrays} * w.max_tiles));
    w.bytes = o;
    return w;
}

}  // namespace

extern "C" int64_t rf_tfr_device_workspace_bytes(const void* blob_host, int32_t batch) {
    if (!blob_host || batch < 0) return -1;
    return plan(*static_cast<const TfrBlobHdr*>(blob_host), batch, nullptr).bytes;
}

extern "C" int rf_tfr_parse_device(const void* blob_dev, const void* blob_host, const uint8_t* rec,
                                   const int64_t* rec_off, int32_t B, int64_t n_rec_bytes, int64_t max_rec_bytes,
                                   const rf_tfr_columns* cols, rf_tfr_dev_stats* stats, void* workspace,
                                   int64_t workspace_bytes, void* stream) {
    if (!blob_dev || !blob_host || !cols || !stats || B <= 0 || !rec || !rec_off || n_rec_bytes < 0 || max_rec_bytes < 0)
        return rf_set_error(RF_EINVAL, "rf_tfr_parse_device: bad argument");
    const TfrBlobHdr& h = *static_cast<const TfrBlobHdr*>(blob_host);
    if (h.F <= 0 || h.F > kMaxFeatures)
        return rf_set_error(RF_EINVAL, "rf_tfr_parse_device: schema of %d features (1..%d supported)", h.F, kMaxFeatures);
    if (n_rec_bytes > INT32_MAX - 16)
        return rf_set_error(RF_EINVAL, "rf_tfr_parse_device: batch of %lld record bytes is too large for int32 offsets",
                            static_cast<long long>(n_rec_bytes));
    const rf_tfr_columns& c = *cols;
    if ((h.Sb && (!c.tok_bytes || !c.tok_off || !c.bag_off || !c.lmax)) || (h.Si && (!c.ival || !c.ibag_off || !c.ilmax)) ||
        (h.Sf && (!c.fval || !c.fbag_off || !c.flmax)) || (h.Ni && !c.iscalar) || (h.Nf && !c.fscalar))
        return rf_set_error(RF_EINVAL, "rf_tfr_parse_device: a column buffer the schema needs is NULL");
    if ((h.Sb && (c.tok_bytes_cap < n_rec_bytes || c.tok_cap < tfr_cap_tok(n_rec_bytes, B, h.Sb))) ||
        (h.Si && c.ival_cap < tfr_cap_ival(n_rec_bytes)) || (h.Sf && c.fval_cap < tfr_cap_fval(n_rec_bytes)))
        return rf_set_error(RF_ENOSPC, "rf_tfr_parse_device: column capacities below the worst case of %lld record bytes",
                            static_cast<long long>(n_rec_bytes));
    Workspace w = plan(h, B, static_cast<uint8_t*>(workspace));
    if (!workspace || workspace_bytes < w.bytes)
        return rf_set_error(RF_EINVAL, "rf_tfr_parse_device: workspace of %lld bytes, need %lld",
                            static_cast<long long>(workspace_bytes), static_cast<long long>(w.bytes));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t* blob = static_cast<const uint8_t*>(blob_dev);

    // LDS: record slot | win[F] | entry list; one wave per workgroup
    const int side = 4 * ((h.F + 3) & ~3) + 12 * kEnt;
    int64_t slot = (max_rec_bytes + 16 + 15) & ~int64_t{15};
    const int64_t slot_cap = (kLdsBudget - side) & ~int64_t{15};
    if (slot > slot_cap) slot = slot_cap;
    if (slot < 0) slot = 0;
    const size_t lds = static_cast<size_t>(slot + side);

    const int gmax = std::max(std::max(h.Sb, h.Si), std::max(h.Sf, 1));
    tfr_init_kernel<<<(gmax + 255) / 256, 256, 0, st>>>(stats, c.lmax, h.Sb, c.ilmax, h.Si, c.flmax, h.Sf);

    CountArgs ca{};
    ca.blob = blob;
    ca.rec = rec;
    ca.rec_off = rec_off;
    ca.B = B;
    ca.slot_bytes = static_cast<int32_t>(slot);
    ca.spans = w.spans;
    ca.tokc = w.tokc;
    ca.tokb = w.tokb;
    ca.ic = w.ic;
    ca.fc = w.fc;
    ca.lmax = c.lmax;
    ca.ilmax = c.ilmax;
    ca.flmax = c.flmax;
    ca.err_rec = w.err_rec;
    ca.stats = stats;
    tfr_count_kernel<<<B, 64, lds, st>>>(ca);

    ScanArgs sa{};
    sa.in[0] = w.tokc;
    sa.out[0] = h.Sb ? c.bag_off : nullptr;
    sa.n[0] = static_cast<int64_t>(B) * h.Sb;
    sa.in[1] = w.tokb;
    sa.out[1] = h.Sb ? w.bstart : nullptr;
    sa.n[1] = static_cast<int64_t>(B) * h.Sb;
    sa.in[2] = w.ic;
    sa.out[2] = h.Si ? c.ibag_off : nullptr;
    sa.n[2] = static_cast<int64_t>(B) * h.Si;
    sa.in[3] = w.fc;
    sa.out[3] = h.Sf ? c.fbag_off : nullptr;
    sa.n[3] = static_cast<int64_t>(B) * h.Sf;
    sa.tsum = w.tsum;
    sa.max_tiles = w.max_tiles;
    sa.stats = stats;
    sa.err_rec = w.err_rec;
    tfr_scan_reduce<<<dim3(w.max_tiles, kScanArrays), 256, 0, st>>>(sa);
    tfr_scan_tiles<<<kScanArrays, 256, 0, st>>>(sa);
    tfr_scan_apply<<<dim3(w.max_tiles, kScanArrays), 256, 0, st>>>(sa);

    WriteArgs wa{};
    wa.blob = blob;
    wa.rec = rec;
    wa.rec_off = rec_off;
    wa.B = B;
    wa.slot_bytes = static_cast<int32_t>(slot);
    wa.spans = w.spans;
    wa.bstart = w.bstart;
    wa.c = c;
    wa.stats = stats;
    tfr_write_kernel<<<B, 64, static_cast<size_t>(slot), st>>>(wa);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rf_set_error(RF_EINVAL, "rf_tfr_parse_device: launch failed: %s", hipGetErrorString(e));
    return RF_OK;
}
