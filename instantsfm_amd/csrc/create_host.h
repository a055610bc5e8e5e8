// Host-side helpers of insfm_ba_create (plain C++, no HIP): a small thread pool that lives for one create call and a
// stable parallel counting sort.  create's structure building is O(N) integer work over a few arrays (camera-major
// lists, the block pattern, the co-visibility graph); done on one core it took ~80 ms for the 2M observations of
// config 3, so every pass over the observations runs on the pool.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace insfm {

// Worker count: INSFM_HOST_THREADS, else the hardware concurrency, capped at 16 (the GPU box's share of host cores).
inline int host_pool_size() {
    static const int hw = [] {
        const char* e = std::getenv("INSFM_HOST_THREADS");
        const int v = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(v, 16));
    }();
    return hw;
}

// Fixed set of threads for the duration of one create call.  run(f) calls f(t) for every t in [0, size()), t = 0 on
// the caller, and returns when all have finished.  Jobs never overlap (one caller).
class HostPool {
  public:
    explicit HostPool(int n) : n_(std::max(1, n)) {
        for (int t = 1; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    int size() const { return n_; }
    void run(const std::function<void(int)>& f) {
        if (n_ == 1) { f(0); return; }
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &f;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
    }
    // f(t, begin, end) over [0, n) in size() contiguous ranges (range t to thread t)
    template <class F>
    void ranges(long long n, F&& f) {
        const long long per = (n + n_ - 1) / n_;
        run([&](int t) {
            const long long a = std::min(n, (long long)t * per), b = std::min(n, a + per);
            if (a < b) f(t, a, b);
        });
    }

  private:
    void loop(int t) {
        long long seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                job = job_;
            }
            (*job)(t);
            {
                std::lock_guard<std::mutex> lk(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    long long gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

// Allocator that leaves new elements uninitialized: create's large index arrays are written in full right after
// they are sized, and value-initializing them first cost a single-threaded pass over ~100 MB.
template <class T>
struct NoInit : std::allocator<T> {
    template <class U>
    struct rebind { using other = NoInit<U>; };
    template <class U>
    void construct(U* p) noexcept { (void)p; }
    template <class U, class... A>
    void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
template <class T>
using nivec = std::vector<T, NoInit<T>>;

// Stable counting sort of the items `items[0..n)` (nullptr: 0..n-1) by key(item) in [0, K): out[ptr[k] ..] lists
// val(item) for the items with key k in their input order; ptr has K + 1 entries.  Each thread counts and scatters one
// contiguous slice of the input.
template <class Key, class Out, class Val>
void pcount_sort(HostPool& pool, long long n, int K, const int* items, Key key, Out& out, std::vector<int>& ptr,
                 Val val) {
    const int T = pool.size();
    std::vector<int> cnt((size_t)T * K, 0);
    pool.ranges(n, [&](int t, long long a, long long b) {
        int* c = cnt.data() + (size_t)t * K;
        for (long long i = a; i < b; ++i) c[key(items ? items[i] : (int)i)]++;
    });
    ptr.assign((size_t)K + 1, 0);
    long long run = 0;
    for (int k = 0; k < K; ++k) {
        ptr[k] = (int)run;
        for (int t = 0; t < T; ++t) {
            const int c = cnt[(size_t)t * K + k];
            cnt[(size_t)t * K + k] = (int)run;
            run += c;
        }
    }
    ptr[K] = (int)run;
    out.resize((size_t)n);
    pool.ranges(n, [&](int t, long long a, long long b) {
        int* c = cnt.data() + (size_t)t * K;
        for (long long i = a; i < b; ++i) {
            const int it = items ? items[i] : (int)i;
            out[c[key(it)]++] = val(it);
        }
    });
}
template <class Key, class Out>
void pcount_sort(HostPool& pool, long long n, int K, const int* items, Key key, Out& out, std::vector<int>& ptr) {
    pcount_sort(pool, n, K, items, key, out, ptr, [](int it) { return it; });
}

}  // namespace insfm
