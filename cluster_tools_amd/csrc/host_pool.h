// host_pool.h — host side of the host-pointer path: a persistent worker pool and the streaming
// (non-temporal) copy / widen loops that move block data between the callers' numpy arrays and
// the pinned staging buffers.
//
// The host path is bound by host memory traffic, not by PCIe or the GPU (r03, config 3: the
// widening of a 13-block batch took longer than its compute).  Two things keep that traffic
// minimal: stores bypass the caches (a regular store to a cold destination line first reads it:
// 8 more bytes per widened voxel), and the threads live across calls (spawning 8 threads per
// block costs more than copying a small block).
#pragma once

#include <emmintrin.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ctws_host {

// parallel_for over [0, n): the calling thread works too; returns when every index is done.
//
// Generations: a worker joins a parallel_for by copying (fn, n) under the lock and counting
// itself active; parallel_for returns only when every index is done AND no worker is still
// inside its claim loop.  So a worker can never carry a claim (next_ index) or a stale fn from
// one generation into the next: next_ / done_ are reset for generation g + 1 only after every
// worker of generation g has left work().
class WorkerPool {
   public:
    explicit WorkerPool(int threads) {
        for (int t = 1; t < threads; ++t) th_.emplace_back([this]() { loop(); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size() + 1; }
    void parallel_for(int64_t n, const std::function<void(int64_t)>& fn) {
        if (n <= 0) return;
        if (th_.empty() || n == 1) {
            for (int64_t i = 0; i < n; ++i) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            done_.store(0);
            ++gen_;
        }
        cv_.notify_all();
        work(&fn, n);
        std::unique_lock<std::mutex> l(m_);
        cv_done_.wait(l, [&]() { return done_.load() >= n_ && active_ == 0; });
        fn_ = nullptr;  // (under the lock: a late worker sees no work and waits for the next gen)
    }

   private:
    void work(const std::function<void(int64_t)>* fn, int64_t n) {
        while (true) {
            const int64_t i = next_.fetch_add(1);
            if (i >= n) return;
            (*fn)(i);
            if (done_.fetch_add(1) + 1 == n) {
                std::lock_guard<std::mutex> g(m_);
                cv_done_.notify_all();
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        while (true) {
            const std::function<void(int64_t)>* fn;
            int64_t n;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&]() { return stop_ || (gen_ != seen && fn_ != nullptr); });
                if (stop_) return;
                seen = gen_;
                fn = fn_;
                n = n_;
                ++active_;
            }
            work(fn, n);
            {
                std::lock_guard<std::mutex> g(m_);
                --active_;
            }
            cv_done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, cv_done_;
    const std::function<void(int64_t)>* fn_ = nullptr;  // guarded by m_
    int64_t n_ = 0;                                     // guarded by m_
    int active_ = 0;                                    // workers inside work(), guarded by m_
    std::atomic<int64_t> next_{0}, done_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// memcpy with streaming stores (the destination is pinned staging the DMA engine reads next)
inline void stream_copy(void* dst, const void* src, size_t n) {
    char* d = (char*)dst;
    const char* s = (const char*)src;
    while (n && ((uintptr_t)d & 15)) {
        *d++ = *s++;
        --n;
    }
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(s + i));
        const __m128i b = _mm_loadu_si128((const __m128i*)(s + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i*)(s + i + 32));
        const __m128i e = _mm_loadu_si128((const __m128i*)(s + i + 48));
        _mm_stream_si128((__m128i*)(d + i), a);
        _mm_stream_si128((__m128i*)(d + i + 16), b);
        _mm_stream_si128((__m128i*)(d + i + 32), c);
        _mm_stream_si128((__m128i*)(d + i + 48), e);
    }
    for (; i + 16 <= n; i += 16) _mm_stream_si128((__m128i*)(d + i), _mm_loadu_si128((const __m128i*)(s + i)));
    if (i < n) std::memcpy(d + i, s + i, n - i);
    _mm_sfence();
}

// o[x] = c[x] + off for x < n, streaming stores
inline void widen_add(uint64_t* o, const uint32_t* c, int64_t n, uint64_t off) {
    int64_t x = 0;
    for (; x < n && ((uintptr_t)(o + x) & 15); ++x) o[x] = (uint64_t)c[x] + off;
    const __m128i vo = _mm_set1_epi64x((long long)off), z = _mm_setzero_si128();
    for (; x + 4 <= n; x += 4) {
        const __m128i v = _mm_loadu_si128((const __m128i*)(c + x));
        _mm_stream_si128((__m128i*)(o + x), _mm_add_epi64(_mm_unpacklo_epi32(v, z), vo));
        _mm_stream_si128((__m128i*)(o + x + 2), _mm_add_epi64(_mm_unpackhi_epi32(v, z), vo));
    }
    for (; x < n; ++x) o[x] = (uint64_t)c[x] + off;
}

// o[x] = c[x] ? c[x] + off : 0 (masked voxels have code 0 and output 0), streaming stores
inline void widen_add_nz(uint64_t* o, const uint32_t* c, int64_t n, uint64_t off) {
    int64_t x = 0;
    for (; x < n && ((uintptr_t)(o + x) & 15); ++x) o[x] = c[x] ? (uint64_t)c[x] + off : 0ull;
    const __m128i vo = _mm_set1_epi64x((long long)off), z = _mm_setzero_si128();
    for (; x + 4 <= n; x += 4) {
        const __m128i v = _mm_loadu_si128((const __m128i*)(c + x));
        const __m128i lo = _mm_unpacklo_epi32(v, z), hi = _mm_unpackhi_epi32(v, z);
        // 64-bit lanes equal to zero: both 32-bit halves zero (SSE2 has no 64-bit compare)
        const __m128i el = _mm_cmpeq_epi32(lo, z), eh = _mm_cmpeq_epi32(hi, z);
        const __m128i ml = _mm_and_si128(el, _mm_shuffle_epi32(el, _MM_SHUFFLE(2, 3, 0, 1)));
        const __m128i mh = _mm_and_si128(eh, _mm_shuffle_epi32(eh, _MM_SHUFFLE(2, 3, 0, 1)));
        _mm_stream_si128((__m128i*)(o + x), _mm_andnot_si128(ml, _mm_add_epi64(lo, vo)));
        _mm_stream_si128((__m128i*)(o + x + 2), _mm_andnot_si128(mh, _mm_add_epi64(hi, vo)));
    }
    for (; x < n; ++x) o[x] = c[x] ? (uint64_t)c[x] + off : 0ull;
}

}  // namespace ctws_host
