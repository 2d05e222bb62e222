// rf_io.cpp — TFRecord(GZIP) <-> batched-CSR feature pipe (include/rf_io.h). Host code only.
//
// Reader: per-file decompression threads (inflate + TFRecord framing with masked CRC-32C; a
// single-member GZIP file is inflated whole by libdeflate when the system has it, zlib streams
// everything else)
// feed a deterministic block_length-1 interleave (tf.data TFRecordDataset(num_parallel_reads),
// backend/core/dataloader.py:567-570); a fork-join parse pool turns a batch of serialized
// tf.train.Example records into the columns parse_example would produce
// (dataloader.py:23-44, 77-89), two passes per example range: (1) locate every schema key and
// count its values, (2) after a prefix sum over ranges, write CSR offsets and values straight into
// the caller's (pinned) buffers. The protobuf wire format is decoded by hand (no libprotobuf).
//
// Writer: tf.io.TFRecordWriter(path, "GZIP") (utils/make_tfrecord.py:142) and the
// tf.train.Example serialisation of build_tfrecord (make_tfrecord.py:94-119).
#include <dlfcn.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rf_io.h"
#include "rf_tfr_blob.h"

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

int rf_set_error(int code, const char* fmt, ...);  // rf_api.cpp

namespace {

// ------------------------------------------------------------------------------------------------
// CRC-32C (Castagnoli). SSE4.2 crc32 instruction when the host has it, slicing-by-8 otherwise.
// ------------------------------------------------------------------------------------------------
struct Crc32cTables {
    uint32_t t[8][256];
    Crc32cTables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
    }
};
const Crc32cTables& crc_tables() {
    static const Crc32cTables tabs;
    return tabs;
}

uint32_t crc32c_sw(uint32_t c, const uint8_t* p, size_t n) {
    const auto& T = crc_tables().t;
    while (n && (reinterpret_cast<uintptr_t>(p) & 7)) { c = (c >> 8) ^ T[0][(c ^ *p++) & 0xff]; --n; }
    while (n >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        w ^= c;
        c = T[7][w & 0xff] ^ T[6][(w >> 8) & 0xff] ^ T[5][(w >> 16) & 0xff] ^ T[4][(w >> 24) & 0xff] ^
            T[3][(w >> 32) & 0xff] ^ T[2][(w >> 40) & 0xff] ^ T[1][(w >> 48) & 0xff] ^ T[0][w >> 56];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xff];
    return c;
}

#if defined(__x86_64__)
// Three interleaved crc32 streams (the instruction's latency is 3 cycles, its throughput 1 a cycle) over blocks
// of kLong / kShort bytes, recombined by "append kLong zero bytes" operators: a GF(2) 32x32 matrix applied
// byte-wise through 4 x 256 tables (M. Adler's crc32c.c construction).
constexpr size_t kCrcLong = 1024, kCrcShort = 128;
uint32_t gf2_times(const uint32_t* mat, uint32_t vec) {
    uint32_t sum = 0;
    for (; vec; vec >>= 1, ++mat)
        if (vec & 1) sum ^= *mat;
    return sum;
}
void gf2_square(uint32_t* sq, const uint32_t* mat) {
    for (int n = 0; n < 32; ++n) sq[n] = gf2_times(mat, mat[n]);
}
struct CrcShift {
    uint32_t t[4][256];
    explicit CrcShift(size_t len) {  // len: a power of two >= 1
        uint32_t even[32], odd[32];
        odd[0] = 0x82F63B78u;
        for (int n = 1; n < 32; ++n) odd[n] = 1u << (n - 1);
        gf2_square(even, odd);  // 2 zero bits
        gf2_square(odd, even);  // 4 zero bits
        const uint32_t* op = even;
        for (;;) {
            gf2_square(even, odd);
            op = even;
            len >>= 1;
            if (!len) break;
            gf2_square(odd, even);
            op = odd;
            len >>= 1;
            if (!len) break;
        }
        for (uint32_t n = 0; n < 256; ++n) {
            t[0][n] = gf2_times(op, n);
            t[1][n] = gf2_times(op, n << 8);
            t[2][n] = gf2_times(op, n << 16);
            t[3][n] = gf2_times(op, n << 24);
        }
    }
    uint32_t operator()(uint32_t c) const { return t[0][c & 0xff] ^ t[1][(c >> 8) & 0xff] ^ t[2][(c >> 16) & 0xff] ^ t[3][c >> 24]; }
};
__attribute__((target("sse4.2"))) uint64_t crc32c_three(uint64_t c0, const uint8_t*& p, size_t& n, size_t blk,
                                                         const CrcShift& sh) {
    while (n >= 3 * blk) {
        uint64_t c1 = 0, c2 = 0;
        for (size_t i = 0; i < blk; i += 8) {
            uint64_t w0, w1, w2;
            std::memcpy(&w0, p + i, 8);
            std::memcpy(&w1, p + blk + i, 8);
            std::memcpy(&w2, p + 2 * blk + i, 8);
            c0 = _mm_crc32_u64(c0, w0);
            c1 = _mm_crc32_u64(c1, w1);
            c2 = _mm_crc32_u64(c2, w2);
        }
        c0 = sh(static_cast<uint32_t>(c0)) ^ static_cast<uint32_t>(c1);
        c0 = sh(static_cast<uint32_t>(c0)) ^ static_cast<uint32_t>(c2);
        p += 3 * blk;
        n -= 3 * blk;
    }
    return c0;
}
__attribute__((target("sse4.2"))) uint32_t crc32c_hw(uint32_t c, const uint8_t* p, size_t n) {
    static const CrcShift shift_long(kCrcLong), shift_short(kCrcShort);
    uint64_t c0 = crc32c_three(c, p, n, kCrcLong, shift_long);
    c0 = crc32c_three(c0, p, n, kCrcShort, shift_short);
    while (n >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        c0 = _mm_crc32_u64(c0, w);
        p += 8;
        n -= 8;
    }
    c = static_cast<uint32_t>(c0);
    while (n--) c = _mm_crc32_u8(c, *p++);
    return c;
}
const bool g_have_sse42 = __builtin_cpu_supports("sse4.2");
#endif

uint32_t crc32c(uint32_t crc, const void* data, size_t n) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    uint32_t c = ~crc;
#if defined(__x86_64__)
    c = g_have_sse42 ? crc32c_hw(c, p, n) : crc32c_sw(c, p, n);
#else
    c = crc32c_sw(c, p, n);
#endif
    return ~c;
}

inline uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

inline uint32_t load_u32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
inline uint64_t load_u64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

struct Status {
    int code = RF_OK;
    std::string msg;
    bool ok() const { return code == RF_OK; }
};
Status fail(int code, std::string msg) { return Status{code, std::move(msg)}; }

// ------------------------------------------------------------------------------------------------
// libdeflate (the system's libdeflate.so.0, loaded at run time; its whole-buffer gzip decoder runs
// ~2-3x zlib's streaming inflate). Only the three entry points the reader needs; absent library or
// RF_TFR_INFLATE=zlib -> zlib for every file.
// ------------------------------------------------------------------------------------------------
struct Deflate {
    using alloc_t = void* (*)();
    using free_t = void (*)(void*);
    // libdeflate_gzip_decompress_ex(d, in, in_n, out, out_avail, &in_used, &out_n) -> 0 success,
    // 1 bad data, 2 short output, 3 insufficient space
    using gunzip_t = int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);
    alloc_t alloc = nullptr;
    free_t release = nullptr;
    gunzip_t gunzip = nullptr;
    Deflate() {
        const char* e = std::getenv("RF_TFR_INFLATE");
        if (e && std::string(e) == "zlib") return;
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = reinterpret_cast<alloc_t>(dlsym(h, "libdeflate_alloc_decompressor"));
        release = reinterpret_cast<free_t>(dlsym(h, "libdeflate_free_decompressor"));
        gunzip = reinterpret_cast<gunzip_t>(dlsym(h, "libdeflate_gzip_decompress_ex"));
        if (!alloc || !release || !gunzip) alloc = nullptr;
    }
    bool ok() const { return alloc != nullptr; }
};
const Deflate& deflate_lib() {
    static const Deflate d;
    return d;
}

// ------------------------------------------------------------------------------------------------
// Byte stream over a file, plain or gzip (concatenated members allowed), read straight into the
// caller's buffer (fread, or inflate with the buffer as its output window).
// ------------------------------------------------------------------------------------------------
class InStream {
  public:
    InStream(const std::string& path, bool gz) : path_(path), gz_(gz) {}
    ~InStream() {
        if (gz_ && z_init_) inflateEnd(&zs_);
        if (f_) std::fclose(f_);
    }
    Status open() {
        f_ = std::fopen(path_.c_str(), "rb");
        if (!f_) return fail(RF_EIO, "cannot open " + path_ + ": " + std::strerror(errno));
        if (gz_ && whole_file()) return {};
        if (gz_) {
            in_.resize(1 << 20);
            std::memset(&zs_, 0, sizeof(zs_));
            if (inflateInit2(&zs_, 16 + MAX_WBITS) != Z_OK) return fail(RF_EIO, "inflateInit2 failed");
            z_init_ = true;
        } else {
            std::setvbuf(f_, nullptr, _IONBF, 0);  // large reads go straight into the chunk
        }
        return {};
    }
    // Fills dst[0, n) as far as the stream allows; *got < n only at the end of the stream.
    Status read(uint8_t* dst, size_t n, size_t* got) {
        *got = 0;
        if (whole_) {
            const size_t k = std::min(n, out_n_ - out_pos_);
            std::memcpy(dst, out_.get() + out_pos_, k);
            out_pos_ += k;
            *got = k;
            return {};
        }
        if (!gz_) {
            while (*got < n) {
                const size_t k = std::fread(dst + *got, 1, n - *got, f_);
                if (k == 0) {
                    if (std::ferror(f_)) return fail(RF_EIO, "read error in " + path_);
                    break;
                }
                *got += k;
            }
            return {};
        }
        while (*got < n) {
            if (zs_.avail_in == 0) {
                const size_t k = std::fread(in_.data(), 1, in_.size(), f_);
                if (k == 0) {
                    if (std::ferror(f_)) return fail(RF_EIO, "read error in " + path_);
                    if (!member_open_) return {};
                    return fail(RF_EDATA, "truncated gzip stream in " + path_);
                }
                zs_.next_in = in_.data();
                zs_.avail_in = static_cast<uInt>(k);
            }
            member_open_ = true;  // a gzip member begins (the first, or one concatenated after a finished one)
            const size_t want = std::min<size_t>(n - *got, 1u << 30);
            zs_.next_out = dst + *got;
            zs_.avail_out = static_cast<uInt>(want);
            const int rc = inflate(&zs_, Z_NO_FLUSH);
            *got += want - zs_.avail_out;
            if (rc == Z_STREAM_END) {
                member_open_ = false;
                if (inflateReset(&zs_) != Z_OK) return fail(RF_EIO, "inflateReset failed");
            } else if (rc != Z_OK && rc != Z_BUF_ERROR) {
                return fail(RF_EDATA, std::string("corrupt gzip stream in ") + path_ + ": " +
                                          (zs_.msg ? zs_.msg : "inflate error"));
            }
        }
        return {};
    }

  private:
    // One gzip member spanning the whole file (what tf.io.TFRecordWriter and this build's writer
    // produce), at most 256 MiB decoded: inflate it in one libdeflate call, sized by the member's
    // ISIZE trailer. Anything else — several members, a bad or truncated stream, no libdeflate — leaves
    // the file to the zlib stream from its first byte, so errors and partial reads are zlib's.
    bool whole_file() {
        const Deflate& lib = deflate_lib();
        if (!lib.ok()) return false;
        if (std::fseek(f_, 0, SEEK_END) != 0) return false;
        const long sz = std::ftell(f_);
        std::rewind(f_);
        if (sz < 18 || sz > (1l << 30)) return false;
        std::unique_ptr<uint8_t[]> in(new uint8_t[static_cast<size_t>(sz)]);  // not zero-initialised
        if (std::fread(in.get(), 1, static_cast<size_t>(sz), f_) != static_cast<size_t>(sz)) {
            std::rewind(f_);
            return false;
        }
        const uint8_t* t = in.get() + sz - 4;
        const size_t isize = static_cast<size_t>(t[0]) | static_cast<size_t>(t[1]) << 8 | static_cast<size_t>(t[2]) << 16 |
                             static_cast<size_t>(t[3]) << 24;
        bool ok = false;
        if (isize <= (256u << 20)) {
            void* d = lib.alloc();
            if (d) {
                std::unique_ptr<uint8_t[]> out(new uint8_t[std::max<size_t>(isize, 1)]);
                huge_pages(out.get(), isize);
                size_t used = 0, n = 0;
                ok = lib.gunzip(d, in.get(), static_cast<size_t>(sz), out.get(), isize, &used, &n) == 0 &&
                     used == static_cast<size_t>(sz) && n == isize;
                lib.release(d);
                if (ok) {
                    out_ = std::move(out);
                    out_n_ = n;
                }
            }
        }
        if (!ok) std::rewind(f_);
        whole_ = ok;
        return ok;
    }

    std::string path_;
    bool gz_;
    FILE* f_ = nullptr;
    z_stream zs_;
    bool z_init_ = false, member_open_ = false;
    std::vector<uint8_t> in_;
    bool whole_ = false;
    std::unique_ptr<uint8_t[]> out_;  // the whole file's decoded bytes (whole_)
    size_t out_n_ = 0, out_pos_ = 0;

  public:
    // whole-file mode: hand the decoded bytes over (the producer frames them in place, no block copies)
    bool take_whole(std::unique_ptr<uint8_t[]>* buf, size_t* n) {
        if (!whole_ || out_pos_ != 0) return false;
        *buf = std::move(out_);
        *n = out_n_;
        out_pos_ = out_n_;
        return true;
    }
    // transparent huge pages for a large decode buffer: 2 MiB faults instead of 4 KiB ones when 16
    // producers fill fresh buffers at once
    static void huge_pages(void* p, size_t n) {
        const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + (2u << 20) - 1) & ~static_cast<uintptr_t>((2u << 20) - 1);
        const uintptr_t e = (reinterpret_cast<uintptr_t>(p) + n) & ~static_cast<uintptr_t>((2u << 20) - 1);
        if (e > a) madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
    }
};

// A block of one file's decoded bytes and the records framed inside it (payloads in place).
struct Chunk {
    std::unique_ptr<uint8_t[]> buf;  // not zero-initialised
    size_t cap = 0;
    std::vector<uint64_t> start;  // record i = buf[start[i], start[i] + len[i])
    std::vector<uint32_t> len;
    explicit Chunk(size_t c) : buf(new uint8_t[c]), cap(c) {}
    Chunk(std::unique_ptr<uint8_t[]> b, size_t c) : buf(std::move(b)), cap(c) {}
    size_t size() const { return start.size(); }
};

// One open file: a thread reads (or inflates) blocks and frames the records inside them into a
// bounded chunk queue.
class FileProducer {
  public:
    FileProducer(std::string path, bool gz) : path_(std::move(path)), gz_(gz) {
        th_ = std::thread([this] { run(); });
    }
    ~FileProducer() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // 1 = record, 0 = end of file, -1 = error (status()).
    int next(const uint8_t** p, uint32_t* n, std::shared_ptr<Chunk>* hold) {
        if (!cur_ || idx_ == cur_->size()) {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [this] { return !q_.empty() || done_; });
            if (q_.empty()) return st_.ok() ? 0 : -1;
            cur_ = std::move(q_.front());
            q_.pop_front();
            idx_ = 0;
            g.unlock();
            cv_.notify_all();
        }
        *p = cur_->buf.get() + cur_->start[idx_];
        *n = cur_->len[idx_];
        *hold = cur_;
        ++idx_;
        return 1;
    }
    const Status& status() const { return st_; }

  private:
    static constexpr size_t kBlockBytes = 4u << 20, kQueueChunks = 6;

    void run() {
        Status s = produce();
        std::lock_guard<std::mutex> g(mu_);
        st_ = s;
        done_ = true;
        cv_.notify_all();
    }
    // Blocks of kBlockBytes; a record cut by the block end moves (with its header) to the front of
    // the next block, which grows when one record needs more than a block.
    Status produce() {
        InStream in(path_, gz_);
        Status s = in.open();
        if (!s.ok()) return s;
        uint64_t rec_no = 0;
        std::shared_ptr<Chunk> chunk;
        size_t have = 0;  // bytes in chunk->buf
        {
            std::unique_ptr<uint8_t[]> whole;
            size_t n = 0;
            if (in.take_whole(&whole, &n)) {  // the decoded file is one chunk; the loop below frames it and sees EOF
                chunk = std::make_shared<Chunk>(std::move(whole), n + 1);
                have = n;
            } else {
                chunk = std::make_shared<Chunk>(kBlockBytes);
            }
        }
        for (;;) {
            size_t got = 0;
            s = in.read(chunk->buf.get() + have, chunk->cap - have, &got);
            if (!s.ok()) return s;
            const bool eof = have + got < chunk->cap;
            have += got;
            const uint8_t* base = chunk->buf.get();
            size_t pos = 0, need = 0;
            while (have - pos >= 12) {
                const uint8_t* h = base + pos;
                const uint64_t len = load_u64(h);
                if (mask_crc(crc32c(0, h, 8)) != load_u32(h + 8))
                    return fail(RF_EDATA, "corrupted record length crc at record " + std::to_string(rec_no) + " of " + path_);
                if (len > (1ull << 31)) return fail(RF_EDATA, "record too large at record " + std::to_string(rec_no) + " of " + path_);
                need = 12 + static_cast<size_t>(len) + 4;
                if (have - pos < need) break;
                if (mask_crc(crc32c(0, h + 12, len)) != load_u32(h + 12 + len))
                    return fail(RF_EDATA, "corrupted record data crc at record " + std::to_string(rec_no) + " of " + path_);
                chunk->start.push_back(pos + 12);
                chunk->len.push_back(static_cast<uint32_t>(len));
                pos += need;
                need = 0;
                ++rec_no;
            }
            const size_t tail = have - pos;
            if (eof) {
                if (tail && tail < 12)
                    return fail(RF_EDATA, "truncated record header at record " + std::to_string(rec_no) + " of " + path_);
                if (tail) return fail(RF_EDATA, "truncated record at record " + std::to_string(rec_no) + " of " + path_);
                if (chunk->size()) push(std::move(chunk));
                return {};
            }
            auto next = std::make_shared<Chunk>(std::max(kBlockBytes, need + (need >> 2)));
            std::memcpy(next->buf.get(), base + pos, tail);
            have = tail;
            if (chunk->size() && !push(std::move(chunk))) return {};
            chunk = std::move(next);
        }
    }
    bool push(std::shared_ptr<Chunk> c) {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return q_.size() < kQueueChunks || stop_; });
        if (stop_) return false;
        q_.push_back(std::move(c));
        cv_.notify_all();
        return true;
    }

    std::string path_;
    bool gz_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Chunk>> q_;
    bool done_ = false, stop_ = false;
    Status st_;
    std::shared_ptr<Chunk> cur_;
    size_t idx_ = 0;
    std::thread th_;
};

// Fork-join pool: run(n, f) calls f(0..n-1) exactly once each, on the workers plus the calling thread.
//
// Every run() is one Job on the caller's stack holding its own function, count and claim counter. A worker
// takes the job pointer and registers itself (active) under the lock, and run() returns only when every index
// is done AND no worker is registered any more, then clears the pointer under the lock. A worker that wakes
// late therefore either finds the job gone (and touches nothing) or holds a registration that keeps the job
// alive: no claim can cross from one run() into the next. (Round 5's pool shared one counter across runs: a
// worker that claimed an index of run N after its end but read run N+1's count executed an index twice and
// let run() return early, with a worker still inside the caller's lambda.)
class Pool {
  public:
    explicit Pool(int n_threads) {
        for (int i = 1; i < n_threads; ++i) ws_.emplace_back([this] { work(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : ws_) t.join();
    }
    int size() const { return static_cast<int>(ws_.size()) + 1; }
    void run(int n, const std::function<void(int)>& f) {
        if (n <= 0) return;
        Job job{&f, n};
        if (n > 1 && !ws_.empty()) {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &job;
            ++gen_;
            cv_.notify_all();
        }
        drain(job);
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return job.done == job.n && job.active == 0; });
        if (job_ == &job) job_ = nullptr;
    }

  private:
    struct Job {
        const std::function<void(int)>* fn;
        int n;
        std::atomic<int> next{0};
        int done = 0;    // indices finished (under mu_)
        int active = 0;  // workers registered on this job (under mu_)
    };
    // claims indices until none is left; counts the finished ones under the lock
    void drain(Job& job) {
        int finished = 0;
        for (;;) {
            const int i = job.next.fetch_add(1);
            if (i >= job.n) break;
            (*job.fn)(i);
            ++finished;
        }
        if (finished) {
            std::lock_guard<std::mutex> g(mu_);
            job.done += finished;
            if (job.done == job.n) done_cv_.notify_all();
        }
    }
    void work() {
        uint64_t seen = 0;
        for (;;) {
            Job* job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
                if (!job) continue;
                ++job->active;
            }
            drain(*job);
            std::lock_guard<std::mutex> g(mu_);
            if (--job->active == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> ws_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    Job* job_ = nullptr;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// ------------------------------------------------------------------------------------------------
// Protobuf wire decoding (tf.train.Example / Features / Feature / {Bytes,Float,Int64}List).
// ------------------------------------------------------------------------------------------------
inline bool get_varint(const uint8_t*& p, const uint8_t* e, uint64_t* v) {
    uint64_t r = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
        const uint8_t b = *p++;
        r |= static_cast<uint64_t>(b & 0x7f) << s;
        if (!(b & 0x80)) { *v = r; return true; }
    }
    return false;
}

// Skips a field of the given wire type; false if malformed.
inline bool skip_field(const uint8_t*& p, const uint8_t* e, uint32_t wt) {
    uint64_t v;
    switch (wt) {
        case 0: return get_varint(p, e, &v);
        case 1: if (e - p < 8) return false; p += 8; return true;
        case 2: if (!get_varint(p, e, &v) || static_cast<uint64_t>(e - p) < v) return false; p += v; return true;
        case 5: if (e - p < 4) return false; p += 4; return true;
        default: return false;
    }
}

// Reads a length-delimited payload span.
inline bool get_span(const uint8_t*& p, const uint8_t* e, const uint8_t** s, uint32_t* n) {
    uint64_t v;
    if (!get_varint(p, e, &v) || static_cast<uint64_t>(e - p) < v) return false;
    *s = p;
    *n = static_cast<uint32_t>(v);
    p += v;
    return true;
}

struct Span {
    const uint8_t* p = nullptr;
    uint32_t n = 0;
    int32_t kind = -1;  // RF_TFR_* of the list, -1 = key absent, -2 = Feature with no kind set
};

// Feature message -> (kind, list span). oneof: the last kind field wins.
inline bool decode_feature(const uint8_t* p, uint32_t n, Span* out) {
    const uint8_t* e = p + n;
    out->kind = -2;
    out->p = nullptr;
    out->n = 0;
    while (p < e) {
        uint64_t tag;
        if (!get_varint(p, e, &tag)) return false;
        const uint32_t field = static_cast<uint32_t>(tag >> 3), wt = tag & 7;
        if (wt == 2 && field >= 1 && field <= 3) {
            if (!get_span(p, e, &out->p, &out->n)) return false;
            out->kind = field == 1 ? RF_TFR_BYTES : field == 2 ? RF_TFR_FLOAT : RF_TFR_INT64;
        } else if (!skip_field(p, e, wt)) {
            return false;
        }
    }
    return true;
}

// Counts the values of a list (and the payload bytes of a BytesList).
inline bool count_list(const Span& s, int64_t* count, int64_t* nbytes) {
    const uint8_t* p = s.p;
    const uint8_t* e = p + s.n;
    int64_t c = 0, b = 0;
    while (p < e) {
        uint64_t tag;
        if (!get_varint(p, e, &tag)) return false;
        const uint32_t field = static_cast<uint32_t>(tag >> 3), wt = tag & 7;
        if (field != 1) {
            if (!skip_field(p, e, wt)) return false;
            continue;
        }
        if (s.kind == RF_TFR_BYTES) {
            if (wt != 2) return false;
            const uint8_t* v;
            uint32_t n;
            if (!get_span(p, e, &v, &n)) return false;
            ++c;
            b += n;
        } else if (s.kind == RF_TFR_FLOAT) {
            if (wt == 5) {
                if (e - p < 4) return false;
                p += 4;
                ++c;
            } else if (wt == 2) {
                const uint8_t* v;
                uint32_t n;
                if (!get_span(p, e, &v, &n) || (n & 3)) return false;
                c += n / 4;
            } else {
                return false;
            }
        } else {
            if (wt == 0) {
                uint64_t v;
                if (!get_varint(p, e, &v)) return false;
                ++c;
            } else if (wt == 2) {
                const uint8_t* v;
                uint32_t n;
                if (!get_span(p, e, &v, &n)) return false;
                const uint8_t* q = v;
                const uint8_t* qe = v + n;
                while (q < qe) {
                    uint64_t x;
                    if (!get_varint(q, qe, &x)) return false;
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

// Writes the values of an already-validated list.
// Returns the byte cursor after the list.
inline int64_t write_bytes(const Span& s, uint8_t* tok_bytes, int32_t* tok_off, int64_t byte_cursor) {
    const uint8_t* p = s.p;
    const uint8_t* e = p + s.n;
    int64_t t = 0;
    while (p < e) {
        uint64_t tag = 0;
        get_varint(p, e, &tag);
        if ((tag >> 3) != 1) { skip_field(p, e, tag & 7); continue; }
        const uint8_t* v = nullptr;
        uint32_t n = 0;
        get_span(p, e, &v, &n);
        std::memcpy(tok_bytes + byte_cursor, v, n);
        tok_off[t++] = static_cast<int32_t>(byte_cursor);
        byte_cursor += n;
    }
    return byte_cursor;
}
inline void write_floats(const Span& s, float* dst) {
    const uint8_t* p = s.p;
    const uint8_t* e = p + s.n;
    while (p < e) {
        uint64_t tag = 0;
        get_varint(p, e, &tag);
        if ((tag >> 3) != 1) { skip_field(p, e, tag & 7); continue; }
        if ((tag & 7) == 5) {
            std::memcpy(dst++, p, 4);
            p += 4;
        } else {
            const uint8_t* v = nullptr;
            uint32_t n = 0;
            get_span(p, e, &v, &n);
            std::memcpy(dst, v, n);
            dst += n / 4;
        }
    }
}
inline void write_int64s(const Span& s, int64_t* dst) {
    const uint8_t* p = s.p;
    const uint8_t* e = p + s.n;
    while (p < e) {
        uint64_t tag = 0;
        get_varint(p, e, &tag);
        if ((tag >> 3) != 1) { skip_field(p, e, tag & 7); continue; }
        uint64_t x = 0;
        if ((tag & 7) == 0) {
            get_varint(p, e, &x);
            *dst++ = static_cast<int64_t>(x);
        } else {
            const uint8_t* v = nullptr;
            uint32_t n = 0;
            get_span(p, e, &v, &n);
            const uint8_t* qe = v + n;
            while (v < qe) {
                get_varint(v, qe, &x);
                *dst++ = static_cast<int64_t>(x);
            }
        }
    }
}

// Compiled schema: map key -> feature index, and each feature's group and position.
struct Schema {
    std::vector<std::string> names;
    std::vector<int32_t> kind, shape, group_pos;  // group_pos: index within its output group
    std::vector<int64_t> def_i;
    std::vector<float> def_f;
    std::unordered_map<std::string_view, int32_t> index;
    int32_t n_bytes = 0, n_iseq = 0, n_fseq = 0, n_iscalar = 0, n_fscalar = 0;

    Status build(const rf_tfr_feature* f, int32_t n) {
        names.reserve(n);
        for (int32_t j = 0; j < n; ++j) {
            if (!f[j].name) return fail(RF_EINVAL, "feature " + std::to_string(j) + " has no name");
            if (f[j].kind < RF_TFR_BYTES || f[j].kind > RF_TFR_FLOAT)
                return fail(RF_EINVAL, std::string("feature ") + f[j].name + ": bad kind");
            if (f[j].shape != RF_TFR_SEQ && f[j].shape != RF_TFR_SCALAR)
                return fail(RF_EINVAL, std::string("feature ") + f[j].name + ": bad shape");
            names.emplace_back(f[j].name);
            kind.push_back(f[j].kind);
            shape.push_back(f[j].shape);
            def_i.push_back(f[j].default_i);
            def_f.push_back(static_cast<float>(f[j].default_f));
            int32_t pos;
            if (f[j].kind == RF_TFR_BYTES) pos = n_bytes++;
            else if (f[j].shape == RF_TFR_SEQ) pos = f[j].kind == RF_TFR_INT64 ? n_iseq++ : n_fseq++;
            else pos = f[j].kind == RF_TFR_INT64 ? n_iscalar++ : n_fscalar++;
            group_pos.push_back(pos);
        }
        for (int32_t j = 0; j < n; ++j) {
            if (!index.emplace(std::string_view(names[j]), j).second)
                return fail(RF_EINVAL, "duplicate feature name " + names[j]);
        }
        return {};
    }
    int32_t size() const { return static_cast<int32_t>(names.size()); }
};

// Locates every schema key of one Example: spans[j] (kind -1 = absent). Last map entry wins.
bool locate(const Schema& sc, const uint8_t* p, uint32_t n, Span* spans) {
    const int32_t F = sc.size();
    for (int32_t j = 0; j < F; ++j) spans[j].kind = -1;
    const uint8_t* e = p + n;
    int32_t guess = 0;
    while (p < e) {  // Example
        uint64_t tag;
        if (!get_varint(p, e, &tag)) return false;
        if (tag != ((1u << 3) | 2)) {
            if (!skip_field(p, e, tag & 7)) return false;
            continue;
        }
        const uint8_t* fs;
        uint32_t fn;
        if (!get_span(p, e, &fs, &fn)) return false;
        const uint8_t* fe = fs + fn;
        while (fs < fe) {  // Features: repeated map entry (field 1)
            if (!get_varint(fs, fe, &tag)) return false;
            if (tag != ((1u << 3) | 2)) {
                if (!skip_field(fs, fe, tag & 7)) return false;
                continue;
            }
            const uint8_t* es;
            uint32_t en;
            if (!get_span(fs, fe, &es, &en)) return false;
            const uint8_t* ee = es + en;
            const uint8_t* key = nullptr;
            uint32_t key_n = 0;
            const uint8_t* val = nullptr;
            uint32_t val_n = 0;
            bool has_val = false;
            while (es < ee) {  // map entry {1: key, 2: Feature}
                uint64_t t2;
                if (!get_varint(es, ee, &t2)) return false;
                if (t2 == ((1u << 3) | 2)) {
                    if (!get_span(es, ee, &key, &key_n)) return false;
                } else if (t2 == ((2u << 3) | 2)) {
                    if (!get_span(es, ee, &val, &val_n)) return false;
                    has_val = true;
                } else if (!skip_field(es, ee, t2 & 7)) {
                    return false;
                }
            }
            // fast path: examples written by one writer list keys in schema order
            int32_t j = -1;
            if (guess < F && sc.names[guess].size() == key_n && std::memcmp(sc.names[guess].data(), key, key_n) == 0) {
                j = guess;
            } else {
                auto it = sc.index.find(std::string_view(reinterpret_cast<const char*>(key), key_n));
                if (it != sc.index.end()) j = it->second;
            }
            if (j < 0) continue;  // not in the feature description: ignored, as parse_example does
            guess = j + 1;
            if (has_val) {
                if (!decode_feature(val, val_n, &spans[j])) return false;
            } else {
                spans[j].kind = -2;
                spans[j].p = nullptr;
                spans[j].n = 0;
            }
        }
    }
    return true;
}

const char* kind_name(int32_t k) { return k == RF_TFR_BYTES ? "bytes" : k == RF_TFR_INT64 ? "int64" : "float"; }

// ------------------------------------------------------------------------------------------------
// Reader
// ------------------------------------------------------------------------------------------------
struct Rec {
    const uint8_t* p;
    uint32_t n;
};

class Reader {
  public:
    Reader(std::vector<std::string> paths, bool gz, int n_threads)
        : paths_(std::move(paths)), gz_(gz), pool_(std::max(1, n_threads)) {
        cycle_.resize(std::max<size_t>(1, std::min<size_t>(paths_.size(), static_cast<size_t>(std::max(1, n_threads)))));
    }

    Status next_batch(const Schema& sc, int32_t batch, rf_tfr_columns* cols) {
        Status s = fill(batch);
        if (!s.ok()) return s;
        const int32_t B = static_cast<int32_t>(std::min<size_t>(batch, pend_.size()));
        s = parse(sc, B, cols);
        if (!s.ok()) return s;
        if (cols->batch == B) {  // consumed: drop the records (and the chunks that held them)
            pend_.erase(pend_.begin(), pend_.begin() + B);
            hold_.erase(hold_.begin(), hold_.begin() + B);
            handed_ += B;
        }
        return {};
    }
    int64_t handed() const { return handed_; }

    // The device-parse host half: the next `batch` records' payloads, packed back to back (rf_io.h).
    Status next_records(int32_t batch, uint8_t* out, int64_t cap, int64_t* rec_off, int32_t* n_out, int64_t* bytes) {
        *n_out = 0;
        *bytes = 0;
        Status s = fill(batch);
        if (!s.ok()) return s;
        const int32_t B = static_cast<int32_t>(std::min<size_t>(batch, pend_.size()));
        int64_t total = 0;
        rec_off[0] = 0;
        for (int32_t b = 0; b < B; ++b) {
            total += pend_[b].n;
            rec_off[b + 1] = total;
        }
        *bytes = total;
        if (total > cap || (total && !out))
            return fail(RF_ENOSPC, "record buffer too small: need " + std::to_string(total) + " bytes, have " +
                                       std::to_string(cap));
        if (B) {
            // ~1 MiB of copying per task
            const int T = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(B, std::min<int64_t>(pool_.size() * 4, total >> 20))));
            pool_.run(T, [&](int t) {
                const int32_t b0 = static_cast<int32_t>(static_cast<int64_t>(B) * t / T);
                const int32_t b1 = static_cast<int32_t>(static_cast<int64_t>(B) * (t + 1) / T);
                for (int32_t b = b0; b < b1; ++b) std::memcpy(out + rec_off[b], pend_[b].p, pend_[b].n);
            });
        }
        pend_.erase(pend_.begin(), pend_.begin() + B);
        hold_.erase(hold_.begin(), hold_.begin() + B);
        handed_ += B;
        *n_out = B;
        return {};
    }

  private:
    // Interleave (tf.data InterleaveDataset order, block_length 1) until `batch` records are pending.
    Status fill(int32_t batch) {
        while (pend_.size() < static_cast<size_t>(batch)) {
            if (!any_open_ && next_path_ >= paths_.size()) return {};
            auto& slot = cycle_[cursor_];
            if (!slot) {
                if (next_path_ < paths_.size()) {
                    // open a file for this slot and for every other empty slot, in the order the cursor reaches
                    // them (the order they would take files one visit at a time), so their producers decode in
                    // parallel instead of each starting only when the round-robin first asks it for a record
                    for (size_t k = 0; k < cycle_.size() && next_path_ < paths_.size(); ++k) {
                        auto& sl = cycle_[(cursor_ + k) % cycle_.size()];
                        if (sl) continue;
                        sl = take_producer();
                        ++n_open_;
                        any_open_ = true;
                    }
                    continue;  // the new file produces in this same turn
                }
                cursor_ = (cursor_ + 1) % cycle_.size();
                continue;
            }
            const uint8_t* p;
            uint32_t n;
            std::shared_ptr<Chunk> hold;
            const int r = slot->next(&p, &n, &hold);
            if (r == 1) {
                pend_.push_back({p, n});
                hold_.push_back(std::move(hold));
                cursor_ = (cursor_ + 1) % cycle_.size();
            } else if (r == 0) {
                slot.reset();
                any_open_ = --n_open_ > 0;
                cursor_ = (cursor_ + 1) % cycle_.size();
            } else {
                Status st = slot->status();
                return st;
            }
        }
        return {};
    }

    // The producer of paths_[next_path_]: files go to slots in path order whatever the slot, so the next
    // cycle_.size() paths are opened ahead (their threads decode while the current files are consumed;
    // a whole-file inflate otherwise stalls its slot at every file boundary).
    std::unique_ptr<FileProducer> take_producer() {
        std::unique_ptr<FileProducer> p;
        if (!ahead_.empty()) {
            p = std::move(ahead_.front());
            ahead_.pop_front();
        } else {
            p = std::make_unique<FileProducer>(paths_[next_path_], gz_);
        }
        ++next_path_;
        // bounded look-ahead: a whole-file inflate holds the compressed file plus its decoded image, so the files
        // opened ahead are capped by a host-memory budget (RF_TFR_AHEAD_MB, default 8192 MiB of on-disk bytes x 5
        // for GZIP) as well as by the cycle length; one file always opens ahead. (1024 MiB bound the cfg2 pipe's
        // 16 x 14 MB files and cost 26 % of the GZIP leg: 0.650 vs 0.877 M ex/s, profiles/r04/pipe_ab.txt)
        const uint64_t budget = ahead_budget();
        uint64_t held = 0;
        for (const auto& a : ahead_) held += a_bytes(a.get());
        while (ahead_.size() < cycle_.size() && next_path_ + ahead_.size() < paths_.size()) {
            const std::string& path = paths_[next_path_ + ahead_.size()];
            const uint64_t need = est_bytes(path);
            if (!ahead_.empty() && held + need > budget) break;
            ahead_.push_back(std::make_unique<FileProducer>(path, gz_));
            ahead_sz_[ahead_.back().get()] = need;
            held += need;
        }
        ahead_sz_.erase(p.get());
        return p;
    }
    uint64_t est_bytes(const std::string& path) const {
        struct stat sb;
        const uint64_t disk = ::stat(path.c_str(), &sb) == 0 ? static_cast<uint64_t>(sb.st_size) : 0;
        return gz_ ? disk * 5 : disk;
    }
    uint64_t a_bytes(const FileProducer* f) const {
        auto it = ahead_sz_.find(f);
        return it == ahead_sz_.end() ? 0 : it->second;
    }
    static uint64_t ahead_budget() {
        static const uint64_t b = [] {
            const char* e = getenv("RF_TFR_AHEAD_MB");
            const long long mb = e ? atoll(e) : 8192;
            return static_cast<uint64_t>(mb > 0 ? mb : 1) << 20;
        }();
        return b;
    }

    Status parse(const Schema& sc, int32_t B, rf_tfr_columns* c) {
        const int32_t F = sc.size();
        c->batch = 0;
        if (B == 0) {
            c->n_tok = c->n_tok_bytes = c->n_ival = c->n_fval = 0;
            return {};
        }
        spans_.resize(static_cast<size_t>(B) * F);
        const int T = std::min(pool_.size() * 4, std::max(1, B / 16));
        struct Part {
            int64_t tok = 0, bytes = 0, ival = 0, fval = 0;
            std::vector<int32_t> lmax;
            Status st;
        };
        std::vector<Part> parts(T);
        const int32_t Sb = sc.n_bytes, Si = sc.n_iseq, Sf = sc.n_fseq;
        auto range = [&](int t, int32_t* b0, int32_t* b1) {
            *b0 = static_cast<int32_t>(static_cast<int64_t>(B) * t / T);
            *b1 = static_cast<int32_t>(static_cast<int64_t>(B) * (t + 1) / T);
        };
        // counts[b*F + j] = value count (bytes: token count); byte totals per (b, j) are not needed
        counts_.resize(static_cast<size_t>(B) * F);
        pool_.run(T, [&](int t) {
            Part& pt = parts[t];
            pt.lmax.assign(static_cast<size_t>(Sb + Si + Sf), 0);
            int32_t b0, b1;
            range(t, &b0, &b1);
            for (int32_t b = b0; b < b1; ++b) {
                Span* sp = &spans_[static_cast<size_t>(b) * F];
                if (!locate(sc, pend_[b].p, pend_[b].n, sp)) {
                    pt.st = fail(RF_EDATA, "malformed tf.train.Example at batch position " + std::to_string(b) +
                                               " (record " + std::to_string(handed_ + b) + ")");
                    return;
                }
                for (int32_t j = 0; j < F; ++j) {
                    Span& s = sp[j];
                    int64_t cnt = 0, nb = 0;
                    if (s.kind >= 0) {
                        if (s.kind != sc.kind[j]) {
                            pt.st = fail(RF_EDATA, "Key: " + sc.names[j] + ". Data types don't match. Expected " +
                                                       kind_name(sc.kind[j]) + ", got " + kind_name(s.kind) +
                                                       " (record " + std::to_string(handed_ + b) + ")");
                            return;
                        }
                        if (!count_list(s, &cnt, &nb)) {
                            pt.st = fail(RF_EDATA, "Key: " + sc.names[j] + ". malformed " + kind_name(s.kind) +
                                                       " list (record " + std::to_string(handed_ + b) + ")");
                            return;
                        }
                    } else if (s.kind == -2) {
                        s.kind = sc.kind[j];  // Feature with no kind: an empty list
                        s.p = nullptr;
                        s.n = 0;
                    }
                    if (sc.shape[j] == RF_TFR_SCALAR) {
                        if (s.kind == -1) {
                            cnt = sc.kind[j] == RF_TFR_BYTES ? 1 : 0;  // missing -> default ("" is one empty token)
                        } else if (cnt != 1) {
                            pt.st = fail(RF_EDATA, "Key: " + sc.names[j] + ". Number of values != expected. Values size: " +
                                                       std::to_string(cnt) + " but output shape: [] (record " +
                                                       std::to_string(handed_ + b) + ")");
                            return;
                        }
                    }
                    if (cnt > INT32_MAX) {
                        pt.st = fail(RF_EDATA, "Key: " + sc.names[j] + ": list too long");
                        return;
                    }
                    counts_[static_cast<size_t>(b) * F + j] = static_cast<int32_t>(cnt);
                    const int32_t g = sc.group_pos[j];
                    if (sc.kind[j] == RF_TFR_BYTES) {
                        pt.tok += cnt;
                        pt.bytes += nb;
                        pt.lmax[g] = std::max<int32_t>(pt.lmax[g], static_cast<int32_t>(cnt));
                    } else if (sc.shape[j] == RF_TFR_SEQ) {
                        if (sc.kind[j] == RF_TFR_INT64) {
                            pt.ival += cnt;
                            pt.lmax[Sb + g] = std::max<int32_t>(pt.lmax[Sb + g], static_cast<int32_t>(cnt));
                        } else {
                            pt.fval += cnt;
                            pt.lmax[Sb + Si + g] = std::max<int32_t>(pt.lmax[Sb + Si + g], static_cast<int32_t>(cnt));
                        }
                    }
                }
            }
        });
        for (auto& pt : parts)
            if (!pt.st.ok()) return pt.st;
        // exclusive scan over ranges
        std::vector<int64_t> tok0(T + 1, 0), bytes0(T + 1, 0), ival0(T + 1, 0), fval0(T + 1, 0);
        for (int t = 0; t < T; ++t) {
            tok0[t + 1] = tok0[t] + parts[t].tok;
            bytes0[t + 1] = bytes0[t] + parts[t].bytes;
            ival0[t + 1] = ival0[t] + parts[t].ival;
            fval0[t + 1] = fval0[t] + parts[t].fval;
        }
        c->n_tok = tok0[T];
        c->n_tok_bytes = bytes0[T];
        c->n_ival = ival0[T];
        c->n_fval = fval0[T];
        if (c->n_tok_bytes > INT32_MAX || c->n_tok > INT32_MAX || c->n_ival > INT32_MAX || c->n_fval > INT32_MAX)
            return fail(RF_EINVAL, "batch too large for int32 CSR offsets; use a smaller batch");
        if (c->n_tok > c->tok_cap || c->n_tok_bytes > c->tok_bytes_cap || c->n_ival > c->ival_cap || c->n_fval > c->fval_cap)
            return fail(RF_ENOSPC, "column capacity too small: need tok " + std::to_string(c->n_tok) + " bytes " +
                                       std::to_string(c->n_tok_bytes) + " ival " + std::to_string(c->n_ival) + " fval " +
                                       std::to_string(c->n_fval));
        if ((Sb && (!c->tok_off || !c->bag_off || !c->lmax || (c->n_tok_bytes && !c->tok_bytes))) ||
            (Si && (!c->ibag_off || !c->ilmax || (c->n_ival && !c->ival))) ||
            (Sf && (!c->fbag_off || !c->flmax || (c->n_fval && !c->fval))) || (sc.n_iscalar && !c->iscalar) ||
            (sc.n_fscalar && !c->fscalar))
            return fail(RF_EINVAL, "a column buffer the schema needs is NULL");
        pool_.run(T, [&](int t) {
            int32_t b0, b1;
            range(t, &b0, &b1);
            int64_t tok = tok0[t], byt = bytes0[t], iv = ival0[t], fv = fval0[t];
            for (int32_t b = b0; b < b1; ++b) {
                const Span* sp = &spans_[static_cast<size_t>(b) * F];
                const int32_t* cn = &counts_[static_cast<size_t>(b) * F];
                for (int32_t j = 0; j < F; ++j) {
                    const int32_t g = sc.group_pos[j];
                    const Span& s = sp[j];
                    const int32_t cnt = cn[j];
                    if (sc.kind[j] == RF_TFR_BYTES) {
                        c->bag_off[static_cast<int64_t>(b) * Sb + g] = static_cast<int32_t>(tok);
                        if (s.kind >= 0) {
                            byt = write_bytes(s, c->tok_bytes, c->tok_off + tok, byt);
                        } else if (cnt == 1) {  // missing SCALAR bytes -> default b""
                            c->tok_off[tok] = static_cast<int32_t>(byt);
                        }
                        tok += cnt;
                    } else if (sc.shape[j] == RF_TFR_SEQ) {
                        if (sc.kind[j] == RF_TFR_INT64) {
                            c->ibag_off[static_cast<int64_t>(b) * Si + g] = static_cast<int32_t>(iv);
                            if (s.kind >= 0) write_int64s(s, c->ival + iv);
                            iv += cnt;
                        } else {
                            c->fbag_off[static_cast<int64_t>(b) * Sf + g] = static_cast<int32_t>(fv);
                            if (s.kind >= 0) write_floats(s, c->fval + fv);
                            fv += cnt;
                        }
                    } else if (sc.kind[j] == RF_TFR_INT64) {
                        int64_t v = sc.def_i[j];
                        if (s.kind >= 0) write_int64s(s, &v);
                        c->iscalar[static_cast<int64_t>(b) * sc.n_iscalar + g] = v;
                    } else {
                        float v = sc.def_f[j];
                        if (s.kind >= 0) write_floats(s, &v);
                        c->fscalar[static_cast<int64_t>(b) * sc.n_fscalar + g] = v;
                    }
                }
            }
        });
        if (Sb) {
            c->bag_off[static_cast<int64_t>(B) * Sb] = static_cast<int32_t>(c->n_tok);
            c->tok_off[c->n_tok] = static_cast<int32_t>(c->n_tok_bytes);
            for (int32_t g = 0; g < Sb; ++g) {
                int32_t m = 0;
                for (auto& pt : parts) m = std::max(m, pt.lmax[g]);
                c->lmax[g] = m;
            }
        }
        if (Si) {
            c->ibag_off[static_cast<int64_t>(B) * Si] = static_cast<int32_t>(c->n_ival);
            for (int32_t g = 0; g < Si; ++g) {
                int32_t m = 0;
                for (auto& pt : parts) m = std::max(m, pt.lmax[Sb + g]);
                c->ilmax[g] = m;
            }
        }
        if (Sf) {
            c->fbag_off[static_cast<int64_t>(B) * Sf] = static_cast<int32_t>(c->n_fval);
            for (int32_t g = 0; g < Sf; ++g) {
                int32_t m = 0;
                for (auto& pt : parts) m = std::max(m, pt.lmax[Sb + Si + g]);
                c->flmax[g] = m;
            }
        }
        c->batch = B;
        return {};
    }

    std::vector<std::string> paths_;
    std::deque<std::unique_ptr<FileProducer>> ahead_;  // opened ahead, in path order
    std::unordered_map<const FileProducer*, uint64_t> ahead_sz_;  // their estimated host bytes
    bool gz_;
    Pool pool_;
    std::vector<std::unique_ptr<FileProducer>> cycle_;
    size_t cursor_ = 0, next_path_ = 0;
    int n_open_ = 0;
    bool any_open_ = false;
    std::vector<Rec> pend_;
    std::vector<std::shared_ptr<Chunk>> hold_;
    std::vector<Span> spans_;
    std::vector<int32_t> counts_;
    int64_t handed_ = 0;
};

// ------------------------------------------------------------------------------------------------
// Writer
// ------------------------------------------------------------------------------------------------
class Writer {
  public:
    Writer(FILE* f, bool gz) : f_(f), gz_(gz) {}
    Status init(int level) {
        if (!gz_) return {};
        std::memset(&zs_, 0, sizeof(zs_));
        if (deflateInit2(&zs_, level, Z_DEFLATED, 16 + MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK)
            return fail(RF_EINVAL, "deflateInit2 failed (level " + std::to_string(level) + ")");
        z_init_ = true;
        out_.resize(1 << 18);
        return {};
    }
    Status write(const uint8_t* p, size_t n) {
        if (failed_) return fail(RF_EIO, "an earlier write failed");
        if (!gz_) {
            if (std::fwrite(p, 1, n, f_) != n) { failed_ = true; return fail(RF_EIO, "fwrite failed"); }
            return {};
        }
        zs_.next_in = const_cast<uint8_t*>(p);
        zs_.avail_in = static_cast<uInt>(n);
        while (zs_.avail_in) {
            Status s = pump(Z_NO_FLUSH);
            if (!s.ok()) return s;
        }
        return {};
    }
    Status close() {
        Status s;
        if (gz_ && z_init_) {
            int rc;
            do {
                zs_.next_out = out_.data();
                zs_.avail_out = static_cast<uInt>(out_.size());
                rc = deflate(&zs_, Z_FINISH);
                const size_t k = out_.size() - zs_.avail_out;
                if (k && std::fwrite(out_.data(), 1, k, f_) != k) failed_ = true;
            } while (rc == Z_OK);
            if (rc != Z_STREAM_END) failed_ = true;
            deflateEnd(&zs_);
            z_init_ = false;
        }
        if (std::fclose(f_) != 0) failed_ = true;
        f_ = nullptr;
        if (failed_) s = fail(RF_EIO, "write/close failed");
        return s;
    }
    ~Writer() {
        if (z_init_) deflateEnd(&zs_);
        if (f_) std::fclose(f_);
    }

  private:
    Status pump(int flush) {
        zs_.next_out = out_.data();
        zs_.avail_out = static_cast<uInt>(out_.size());
        const int rc = deflate(&zs_, flush);
        if (rc == Z_STREAM_ERROR) { failed_ = true; return fail(RF_EIO, "deflate failed"); }
        const size_t k = out_.size() - zs_.avail_out;
        if (k && std::fwrite(out_.data(), 1, k, f_) != k) { failed_ = true; return fail(RF_EIO, "fwrite failed"); }
        return {};
    }
    FILE* f_;
    bool gz_;
    z_stream zs_;
    bool z_init_ = false, failed_ = false;
    std::vector<uint8_t> out_;
};

// ------------------------------------------------------------------------------------------------
// Example encoding
// ------------------------------------------------------------------------------------------------
inline size_t varint_size(uint64_t v) {
    size_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}
inline uint8_t* put_varint(uint8_t* p, uint64_t v) {
    while (v >= 0x80) { *p++ = static_cast<uint8_t>(v | 0x80); v >>= 7; }
    *p++ = static_cast<uint8_t>(v);
    return p;
}

struct ListView {  // one (example, feature) value list of the input columns
    int32_t kind;
    int64_t begin, end;  // element range in its group's value array (bytes: token range)
    int64_t scalar_i;
    float scalar_f;
    bool scalar;
};

struct Encoder {
    const Schema& sc;
    const rf_tfr_columns& c;

    ListView view(int32_t b, int32_t j) const {
        ListView v{sc.kind[j], 0, 0, 0, 0.f, false};
        const int32_t g = sc.group_pos[j];
        if (sc.kind[j] == RF_TFR_BYTES) {
            v.begin = c.bag_off[static_cast<int64_t>(b) * sc.n_bytes + g];
            v.end = c.bag_off[static_cast<int64_t>(b) * sc.n_bytes + g + 1];
        } else if (sc.shape[j] == RF_TFR_SEQ) {
            const int32_t* bo = sc.kind[j] == RF_TFR_INT64 ? c.ibag_off : c.fbag_off;
            const int32_t S = sc.kind[j] == RF_TFR_INT64 ? sc.n_iseq : sc.n_fseq;
            v.begin = bo[static_cast<int64_t>(b) * S + g];
            v.end = bo[static_cast<int64_t>(b) * S + g + 1];
        } else {
            v.scalar = true;
            if (sc.kind[j] == RF_TFR_INT64) v.scalar_i = c.iscalar[static_cast<int64_t>(b) * sc.n_iscalar + g];
            else v.scalar_f = c.fscalar[static_cast<int64_t>(b) * sc.n_fscalar + g];
        }
        return v;
    }
    // payload size of the {Bytes,Float,Int64}List message
    size_t list_size(const ListView& v) const {
        if (v.kind == RF_TFR_BYTES) {
            size_t s = 0;
            for (int64_t t = v.begin; t < v.end; ++t) {
                const uint64_t n = static_cast<uint64_t>(c.tok_off[t + 1] - c.tok_off[t]);
                s += 1 + varint_size(n) + n;
            }
            return s;
        }
        if (v.kind == RF_TFR_FLOAT) {
            const uint64_t n = v.scalar ? 1 : static_cast<uint64_t>(v.end - v.begin);
            return n ? 1 + varint_size(4 * n) + 4 * n : 0;
        }
        uint64_t n = 0;
        if (v.scalar) n = varint_size(static_cast<uint64_t>(v.scalar_i));
        else for (int64_t t = v.begin; t < v.end; ++t) n += varint_size(static_cast<uint64_t>(c.ival[t]));
        const bool empty = v.scalar ? false : v.end == v.begin;
        return empty ? 0 : 1 + varint_size(n) + n;
    }
    uint8_t* put_list(uint8_t* p, const ListView& v) const {
        if (v.kind == RF_TFR_BYTES) {
            for (int64_t t = v.begin; t < v.end; ++t) {
                const uint64_t n = static_cast<uint64_t>(c.tok_off[t + 1] - c.tok_off[t]);
                *p++ = 0x0a;
                p = put_varint(p, n);
                std::memcpy(p, c.tok_bytes + c.tok_off[t], n);
                p += n;
            }
            return p;
        }
        if (v.kind == RF_TFR_FLOAT) {
            const uint64_t n = v.scalar ? 1 : static_cast<uint64_t>(v.end - v.begin);
            if (!n) return p;
            *p++ = 0x0a;
            p = put_varint(p, 4 * n);
            const float* src = v.scalar ? &v.scalar_f : c.fval + v.begin;
            std::memcpy(p, src, 4 * n);
            return p + 4 * n;
        }
        if (!v.scalar && v.end == v.begin) return p;
        uint64_t n = 0;
        if (v.scalar) n = varint_size(static_cast<uint64_t>(v.scalar_i));
        else for (int64_t t = v.begin; t < v.end; ++t) n += varint_size(static_cast<uint64_t>(c.ival[t]));
        *p++ = 0x0a;
        p = put_varint(p, n);
        if (v.scalar) return put_varint(p, static_cast<uint64_t>(v.scalar_i));
        for (int64_t t = v.begin; t < v.end; ++t) p = put_varint(p, static_cast<uint64_t>(c.ival[t]));
        return p;
    }
    // Feature = {field kind+1... : list}; entry = {1: key, 2: Feature}
    size_t feature_size(const ListView& v) const {
        const size_t l = list_size(v);
        return 1 + varint_size(l) + l;
    }
    size_t entry_size(int32_t j, const ListView& v) const {
        const size_t k = sc.names[j].size(), f = feature_size(v);
        return 1 + varint_size(k) + k + 1 + varint_size(f) + f;
    }
    size_t features_size(int32_t b) const {
        size_t s = 0;
        for (int32_t j = 0; j < sc.size(); ++j) {
            const size_t e = entry_size(j, view(b, j));
            s += 1 + varint_size(e) + e;
        }
        return s;
    }
    size_t example_size(int32_t b) const {
        const size_t f = features_size(b);
        return 1 + varint_size(f) + f;
    }
    uint8_t* put_example(uint8_t* p, int32_t b) const {
        *p++ = 0x0a;
        p = put_varint(p, features_size(b));
        for (int32_t j = 0; j < sc.size(); ++j) {
            const ListView v = view(b, j);
            *p++ = 0x0a;
            p = put_varint(p, entry_size(j, v));
            *p++ = 0x0a;
            p = put_varint(p, sc.names[j].size());
            std::memcpy(p, sc.names[j].data(), sc.names[j].size());
            p += sc.names[j].size();
            *p++ = 0x12;
            p = put_varint(p, feature_size(v));
            *p++ = static_cast<uint8_t>(v.kind == RF_TFR_BYTES ? 0x0a : v.kind == RF_TFR_FLOAT ? 0x12 : 0x1a);
            p = put_varint(p, list_size(v));
            p = put_list(p, v);
        }
        return p;
    }
};

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" uint32_t rf_crc32c(uint32_t crc, const void* data, size_t n) { return crc32c(crc, data, n); }

extern "C" uint32_t rf_crc32c_masked(const void* data, size_t n) { return mask_crc(crc32c(0, data, n)); }

extern "C" int rf_tfw_open(const char* path, int32_t compression, int32_t level, void** out_writer) {
    if (!path || !out_writer) return rf_set_error(RF_EINVAL, "rf_tfw_open: NULL argument");
    if (compression != RF_TFR_NONE && compression != RF_TFR_GZIP)
        return rf_set_error(RF_EINVAL, "rf_tfw_open: compression must be RF_TFR_NONE or RF_TFR_GZIP");
    if (level < -1 || level > 9) return rf_set_error(RF_EINVAL, "rf_tfw_open: level must be -1..9");
    *out_writer = nullptr;
    FILE* f = std::fopen(path, "wb");
    if (!f) return rf_set_error(RF_EIO, "rf_tfw_open: cannot open %s: %s", path, std::strerror(errno));
    auto* w = new (std::nothrow) Writer(f, compression == RF_TFR_GZIP);
    if (!w) {
        std::fclose(f);
        return rf_set_error(RF_EIO, "rf_tfw_open: out of memory");
    }
    Status s = w->init(level);
    if (!s.ok()) {
        delete w;
        return rf_set_error(s.code, "rf_tfw_open: %s", s.msg.c_str());
    }
    *out_writer = w;
    return RF_OK;
}

extern "C" int rf_tfw_write(void* writer, const void* record, int64_t len) {
    if (!writer || (len && !record) || len < 0) return rf_set_error(RF_EINVAL, "rf_tfw_write: bad argument");
    auto* w = static_cast<Writer*>(writer);
    uint8_t hdr[12];
    const uint64_t n = static_cast<uint64_t>(len);
    std::memcpy(hdr, &n, 8);
    const uint32_t hc = mask_crc(crc32c(0, hdr, 8));
    std::memcpy(hdr + 8, &hc, 4);
    const uint32_t dc = mask_crc(crc32c(0, record, static_cast<size_t>(len)));
    Status s = w->write(hdr, 12);
    if (s.ok() && len) s = w->write(static_cast<const uint8_t*>(record), static_cast<size_t>(len));
    if (s.ok()) s = w->write(reinterpret_cast<const uint8_t*>(&dc), 4);
    if (!s.ok()) return rf_set_error(s.code, "rf_tfw_write: %s", s.msg.c_str());
    return RF_OK;
}

extern "C" int rf_tfw_close(void* writer) {
    if (!writer) return rf_set_error(RF_EINVAL, "rf_tfw_close: NULL writer");
    auto* w = static_cast<Writer*>(writer);
    Status s = w->close();
    delete w;
    if (!s.ok()) return rf_set_error(s.code, "rf_tfw_close: %s", s.msg.c_str());
    return RF_OK;
}

extern "C" int rf_tfr_encode_examples(const rf_tfr_feature* feats, int32_t n_feats, const rf_tfr_columns* cols,
                                      uint8_t* out, int64_t out_cap, int64_t* rec_off, int64_t* needed) {
    if (!feats || n_feats <= 0 || !cols || !rec_off || !needed || cols->batch < 0)
        return rf_set_error(RF_EINVAL, "rf_tfr_encode_examples: bad argument");
    Schema sc;
    Status s = sc.build(feats, n_feats);
    if (!s.ok()) return rf_set_error(s.code, "rf_tfr_encode_examples: %s", s.msg.c_str());
    const rf_tfr_columns& c = *cols;
    if ((sc.n_bytes && (!c.bag_off || !c.tok_off)) || (sc.n_iseq && !c.ibag_off) || (sc.n_fseq && !c.fbag_off) ||
        (sc.n_iscalar && !c.iscalar) || (sc.n_fscalar && !c.fscalar))
        return rf_set_error(RF_EINVAL, "rf_tfr_encode_examples: a column buffer the schema needs is NULL");
    Encoder enc{sc, c};
    int64_t total = 0;
    rec_off[0] = 0;
    for (int32_t b = 0; b < c.batch; ++b) {
        total += static_cast<int64_t>(enc.example_size(b));
        rec_off[b + 1] = total;
    }
    *needed = total;
    if (total > out_cap || (total && !out))
        return rf_set_error(RF_ENOSPC, "rf_tfr_encode_examples: need %lld bytes, have %lld", (long long)total,
                            (long long)out_cap);
    for (int32_t b = 0; b < c.batch; ++b) {
        uint8_t* e = enc.put_example(out + rec_off[b], b);
        if (e != out + rec_off[b + 1]) return rf_set_error(RF_EINVAL, "rf_tfr_encode_examples: internal size mismatch");
    }
    return RF_OK;
}

extern "C" int rf_tfr_open(const char* const* paths, int32_t n_paths, int32_t compression, int32_t n_threads,
                           void** out_reader) {
    if (!paths || n_paths <= 0 || !out_reader) return rf_set_error(RF_EINVAL, "rf_tfr_open: need at least one path");
    if (compression != RF_TFR_NONE && compression != RF_TFR_GZIP)
        return rf_set_error(RF_EINVAL, "rf_tfr_open: compression must be RF_TFR_NONE or RF_TFR_GZIP");
    if (n_threads <= 0 || n_threads > 256) return rf_set_error(RF_EINVAL, "rf_tfr_open: n_threads must be 1..256");
    std::vector<std::string> ps;
    for (int32_t i = 0; i < n_paths; ++i) {
        if (!paths[i]) return rf_set_error(RF_EINVAL, "rf_tfr_open: path %d is NULL", i);
        FILE* f = std::fopen(paths[i], "rb");  // fail at open time, as TFRecordDataset does on iteration
        if (!f) return rf_set_error(RF_EIO, "rf_tfr_open: cannot open %s: %s", paths[i], std::strerror(errno));
        std::fclose(f);
        ps.emplace_back(paths[i]);
    }
    *out_reader = new Reader(std::move(ps), compression == RF_TFR_GZIP, n_threads);
    return RF_OK;
}

extern "C" int rf_tfr_next_batch(void* reader, const rf_tfr_feature* feats, int32_t n_feats, int32_t batch,
                                 rf_tfr_columns* cols) {
    if (!reader || !feats || n_feats <= 0 || !cols || batch <= 0 || cols->reserved != 0)
        return rf_set_error(RF_EINVAL, "rf_tfr_next_batch: bad argument");
    Schema sc;
    Status s = sc.build(feats, n_feats);
    if (s.ok()) s = static_cast<Reader*>(reader)->next_batch(sc, batch, cols);
    if (!s.ok()) return rf_set_error(s.code, "rf_tfr_next_batch: %s", s.msg.c_str());
    return RF_OK;
}

extern "C" int rf_tfr_next_records(void* reader, int32_t batch, uint8_t* out, int64_t out_cap, int64_t* rec_off,
                                   int32_t* n_records, int64_t* n_bytes) {
    if (!reader || batch <= 0 || !rec_off || !n_records || !n_bytes || out_cap < 0)
        return rf_set_error(RF_EINVAL, "rf_tfr_next_records: bad argument");
    Status s = static_cast<Reader*>(reader)->next_records(batch, out, out_cap, rec_off, n_records, n_bytes);
    if (!s.ok()) return rf_set_error(s.code, "rf_tfr_next_records: %s", s.msg.c_str());
    return RF_OK;
}

extern "C" int rf_tfr_schema_blob(const rf_tfr_feature* feats, int32_t n_feats, void* out, int64_t out_cap,
                                  int64_t* needed) {
    if (!feats || n_feats <= 0 || !needed) return rf_set_error(RF_EINVAL, "rf_tfr_schema_blob: bad argument");
    Schema sc;
    Status s = sc.build(feats, n_feats);
    if (!s.ok()) return rf_set_error(s.code, "rf_tfr_schema_blob: %s", s.msg.c_str());
    int32_t hsize = 1;
    while (hsize < 2 * n_feats) hsize <<= 1;
    int64_t names = 0;
    for (auto& nm : sc.names) names += static_cast<int64_t>(nm.size());
    const int64_t names_off = static_cast<int64_t>(sizeof(TfrBlobHdr)) + static_cast<int64_t>(sizeof(TfrBlobFeat)) * n_feats +
                              4 * static_cast<int64_t>(hsize);
    const int64_t total = (names_off + names + 15) & ~int64_t{15};
    *needed = total;
    if (names_off + names > INT32_MAX) return rf_set_error(RF_EINVAL, "rf_tfr_schema_blob: schema too large");
    if (!out || out_cap < total)
        return rf_set_error(RF_ENOSPC, "rf_tfr_schema_blob: need %lld bytes", static_cast<long long>(total));
    auto* base = static_cast<uint8_t*>(out);
    std::memset(base, 0, static_cast<size_t>(total));
    TfrBlobHdr h{};
    h.F = n_feats;
    h.Sb = sc.n_bytes;
    h.Si = sc.n_iseq;
    h.Sf = sc.n_fseq;
    h.Ni = sc.n_iscalar;
    h.Nf = sc.n_fscalar;
    h.hmask = hsize - 1;
    h.names_off = static_cast<int32_t>(names_off);
    h.total_bytes = total;
    std::memcpy(base, &h, sizeof(h));
    auto* fe = reinterpret_cast<TfrBlobFeat*>(base + sizeof(TfrBlobHdr));
    auto* ht = reinterpret_cast<int32_t*>(base + sizeof(TfrBlobHdr) + sizeof(TfrBlobFeat) * n_feats);
    for (int32_t i = 0; i < hsize; ++i) ht[i] = -1;
    int64_t no = 0;
    for (int32_t j = 0; j < n_feats; ++j) {
        TfrBlobFeat f{};
        f.kind = sc.kind[j];
        f.shape = sc.shape[j];
        f.gpos = sc.group_pos[j];
        f.name_off = static_cast<int32_t>(no);
        f.name_len = static_cast<int32_t>(sc.names[j].size());
        f.def_i = sc.def_i[j];
        f.def_f = sc.def_f[j];
        fe[j] = f;
        std::memcpy(base + names_off + no, sc.names[j].data(), sc.names[j].size());
        no += f.name_len;
        uint32_t slot = tfr_key_hash_host(reinterpret_cast<const uint8_t*>(sc.names[j].data()),
                                          static_cast<uint32_t>(sc.names[j].size())) & static_cast<uint32_t>(hsize - 1);
        while (ht[slot] >= 0) slot = (slot + 1) & static_cast<uint32_t>(hsize - 1);
        ht[slot] = j;
    }
    return RF_OK;
}

extern "C" int rf_tfr_device_check(const rf_tfr_dev_stats* st, const rf_tfr_feature* feats, int32_t n_feats,
                                   int64_t first_record) {
    if (!st || !feats || n_feats <= 0) return rf_set_error(RF_EINVAL, "rf_tfr_device_check: bad argument");
    if (st->err_b == INT32_MAX) return RF_OK;
    const int64_t rec = first_record + st->err_b;
    const int32_t j = st->err_feat;
    if (st->err_type != 1 && (j < 0 || j >= n_feats || !feats[j].name))
        return rf_set_error(RF_EDATA, "rf_tfr_next_batch: parse error %d at record %lld", st->err_type, (long long)rec);
    std::string m;
    switch (st->err_type) {  // the texts of Reader::parse
        case 1:
            m = "malformed tf.train.Example at batch position " + std::to_string(st->err_b) + " (record " +
                std::to_string(rec) + ")";
            break;
        case 2:
            m = std::string("Key: ") + feats[j].name + ". Data types don't match. Expected " + kind_name(feats[j].kind) +
                ", got " + kind_name(st->err_kind) + " (record " + std::to_string(rec) + ")";
            break;
        case 3:
            m = std::string("Key: ") + feats[j].name + ". malformed " + kind_name(feats[j].kind) + " list (record " +
                std::to_string(rec) + ")";
            break;
        default:
            m = std::string("Key: ") + feats[j].name + ". Number of values != expected. Values size: " +
                std::to_string(st->err_count) + " but output shape: [] (record " + std::to_string(rec) + ")";
    }
    return rf_set_error(RF_EDATA, "rf_tfr_next_batch: %s", m.c_str());
}

extern "C" int64_t rf_tfr_records_read(void* reader) {
    return reader ? static_cast<Reader*>(reader)->handed() : -1;
}

extern "C" int rf_tfr_close(void* reader) {
    if (!reader) return rf_set_error(RF_EINVAL, "rf_tfr_close: NULL reader");
    delete static_cast<Reader*>(reader);
    return RF_OK;
}
