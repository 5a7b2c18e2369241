// Output files of the reference program (SpeedUp:725-1032, `%lg` text) written off the time loop.
//
// The reference formats every number with fprintf("%lg") on the simulation thread, so at the
// reference cadence (output() every sampleFreq MD steps, writeConditions at the end) text
// formatting is most of an MD interval at N = 3.5k.  Here:
//   * LgText formats with std::to_chars(general, precision 6), which is specified to produce
//     exactly printf("%.6g") in the C locale (= "%lg") — same bytes, several times faster; non-
//     finite values go through snprintf so "inf"/"-nan" spellings stay glibc's;
//   * FileWriter formats and writes whole files on a few background threads from snapshots the
//     caller hands over, so the device keeps stepping while the text is produced (SURVEY §8(f)1,
//     "async writers").  flush() is the only join point: the engine calls it before anything
//     reads the files back (readConditions), at the end of mdqt_run and in mdqt_destroy, and
//     reports the first I/O error there.
#pragma once

#include <cerrno>
#include <charconv>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace mdqt {

// "%lg" text into a growing buffer, spilled to the FILE every ~1 MB (bounded memory at N = 1M)
class LgText {
  public:
    explicit LgText(FILE* f = nullptr) : f_(f) { s_.reserve(kSpill + 4096); }
    ~LgText() { spill(); }
    void num(double x) {
        char b[40];
        if (std::isfinite(x)) {
            auto r = std::to_chars(b, b + sizeof b, x, std::chars_format::general, 6);
            s_.append(b, r.ptr - b);
        } else {
            int n = snprintf(b, sizeof b, "%lg", x);
            s_.append(b, n);
        }
        if (s_.size() >= kSpill) spill();
    }
    void integer(long long v) {
        char b[24];
        auto r = std::to_chars(b, b + sizeof b, v);
        s_.append(b, r.ptr - b);
    }
    void ch(char c) { s_.push_back(c); }
    void str(const char* p) { s_.append(p); }
    const std::string& text() const { return s_; }   // (no FILE: the whole text, for tests)
    bool ok() const { return ok_; }
    void spill() {
        if (!f_ || s_.empty()) return;
        if (fwrite(s_.data(), 1, s_.size(), f_) != s_.size()) ok_ = false;
        s_.clear();
    }

  private:
    static constexpr size_t kSpill = 1 << 20;
    FILE* f_;
    std::string s_;
    bool ok_ = true;
};

class FileWriter {
  public:
    using Fill = std::function<void(LgText&)>;

    explicit FileWriter(int threads = 4) {
        if (threads < 1) threads = 1;
        for (int i = 0; i < threads; ++i) pool_.emplace_back([this] { loop(); });
    }
    ~FileWriter() {
        flush(nullptr);
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : pool_) t.join();
    }
    FileWriter(const FileWriter&) = delete;
    FileWriter& operator=(const FileWriter&) = delete;

    // format and write `path` (mode "w" or "a") on a pool thread; `fill` owns its data
    void submit(std::string path, const char* mode, Fill fill) {
        {
            std::lock_guard<std::mutex> g(m_);
            q_.push_back(Job{std::move(path), mode, std::move(fill)});
            ++pending_;
        }
        cv_.notify_one();
    }

    // wait until every submitted file is on disk; 0, or -1 with the first error in *err
    int flush(std::string* err) {
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
        if (err_.empty()) return 0;
        if (err) *err = err_;
        err_.clear();
        return -1;
    }

  private:
    struct Job {
        std::string path;
        const char* mode;
        Fill fill;
    };

    void loop() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                j = std::move(q_.front());
                q_.pop_front();
            }
            std::string e;
            FILE* f = fopen(j.path.c_str(), j.mode);
            if (!f) {
                e = "cannot open " + j.path + ": " + strerror(errno);
            } else {
                bool ok;
                {
                    LgText t(f);
                    j.fill(t);
                    t.spill();
                    ok = t.ok();
                }
                if (fclose(f) != 0 || !ok) e = "write error on " + j.path;
            }
            j.fill = nullptr;                  // release the snapshot before signalling
            {
                std::lock_guard<std::mutex> g(m_);
                if (!e.empty() && err_.empty()) err_ = e;
                if (--pending_ == 0) done_.notify_all();
            }
        }
    }

    std::mutex m_;
    std::condition_variable cv_, done_;
    std::deque<Job> q_;
    std::vector<std::thread> pool_;
    size_t pending_ = 0;
    bool stop_ = false;
    std::string err_;
};

}  // namespace mdqt
