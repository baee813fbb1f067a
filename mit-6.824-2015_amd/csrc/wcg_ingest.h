// wcg_ingest.h - host side of the GPU Split (mapreduce.go:141-179): input bytes reach HBM in
// line-aligned chunks through two pinned staging buffers, so the PCIe copy of chunk k + 1 and the
// host read of chunk k + 2 overlap the map kernels of chunk k.
//
//   reader threads (a small pool) fill pinned buffer k % 2 from the source (pread of a file, or
//   memcpy of a pageable host split) and scan their slice for '\n' as they go;
//   the chunk is cut after its last '\n' (a partial line moves to the front of the next buffer),
//   so no line, token or rune straddles a chunk;
//   Split's 64 KiB line limit (quirk P1) is emulated: the first line that does not fit
//   bufio.Scanner's buffer with its '\n' ends the input, as it ends the reference's scan;
//   the copy stream waits until device buffer k % 2 is free (its previous map kernels are done),
//   copies, and the map stream waits for the copy.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "wcg_scan.h"

namespace wcg {

// staging slots (pinned host + device buffer pairs): three, so that the reader threads can run a
// chunk ahead of the copy when a read is slow (two kept the copy engine idle between copies)
constexpr int INGEST_SLOTS = 3;

// One thread that issues the chunks' copies and map launches in order (r04).  hipMemcpyAsync from
// pinned memory returned only once the 64 MiB copy was done (rocprofv3 memory-copy trace of
// wcg_map_file: the copy engine sat idle while the calling thread read the next chunk, 1.55 ms per
// chunk against 1.27 ms of copy), so the issuing moved off the thread that reads.
class Issuer {
  public:
    explicit Issuer(std::function<int(int, uint64_t)> issue) : issue_(std::move(issue)), th_([this] { loop(); }) {}
    ~Issuer() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // queue chunk (slot, bytes); the slot's staging buffer belongs to the issuer until released
    void push(int slot, uint64_t n) {
        std::lock_guard<std::mutex> g(m_);
        q_.push_back({slot, n});
        busy_[slot] = true;
        cv_.notify_all();
    }
    // wait until the slot's staging buffer has been copied (and may be refilled); first error
    int wait_slot(int slot) {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return !busy_[slot] || rc_ != 0; });
        return rc_;
    }
    int drain() {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] {
            for (bool b : busy_) if (b) return false;
            return q_.empty();
        });
        return rc_;
    }

  private:
    struct Item { int slot; uint64_t n; };
    void loop() {
        std::unique_lock<std::mutex> g(m_);
        while (true) {
            cv_.wait(g, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;
            const Item it = q_.front();
            q_.erase(q_.begin());
            g.unlock();
            const int rc = rc_ ? rc_ : issue_(it.slot, it.n);   // returns once the staging copy is done
            g.lock();
            if (rc && !rc_) rc_ = rc;
            busy_[it.slot] = false;
            cv_.notify_all();
        }
    }
    std::function<int(int, uint64_t)> issue_;
    std::mutex m_;
    std::condition_variable cv_;
    std::vector<Item> q_;
    bool busy_[INGEST_SLOTS] = {};
    bool stop_ = false;
    int rc_ = 0;
    std::thread th_;
};

// fixed pool of worker threads running one batch of indexed tasks at a time
class TaskPool {
  public:
    explicit TaskPool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this, i] { loop(i); });
    }
    ~TaskPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    // run f(0..n-1) on the pool and wait for all of them
    void run(int n, const std::function<void(int)>& f) {
        std::unique_lock<std::mutex> g(m_);
        f_ = &f;
        ntask_ = n;
        next_ = 0;
        done_ = 0;
        gen_++;
        cv_.notify_all();
        done_cv_.wait(g, [&] { return done_ == ntask_; });
        f_ = nullptr;
    }

  private:
    void loop(int) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(m_);
        while (true) {
            cv_.wait(g, [&] { return gen_ != seen; });
            seen = gen_;
            if (stop_) return;
            while (f_ && next_ < ntask_) {
                const int t = next_++;
                const std::function<void(int)>* f = f_;
                g.unlock();
                (*f)(t);
                g.lock();
                if (++done_ == ntask_) done_cv_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* f_ = nullptr;
    int ntask_ = 0, next_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace wcg
