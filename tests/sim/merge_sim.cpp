// merge_sim.cpp — CPU model of k_cg_fit's drain-merge protocol (test infrastructure, not product code).
//
// The decision logic of the merge block in spark-timeseries_amd/csrc/arima_kernels_impl.hpp (k_cg_fit, "Drain
// merge"), restated with std::atomic on host threads: one thread per bulk wave, one packed word
//   ctl40 = (entries reserved << 24) | active waves,   ctl41 = entries claimed,
// pool entries written, then their ready words (release), read after the ready word (acquire). Each wave holds up to
// SPW slots; a slot's series needs a random number of passes. Waves refill from a shared work counter until it runs
// out; then, as on the device: a wave with 0 < live <= T offers its live slots (reserve + leave the active count in
// one CAS, only while another wave is active and the pool has room), a wave with room claims reserved entries (up to
// 64 live), and a wave with nothing live leaves only by a CAS that sees every reserved entry claimed.
//
// Checked: every series is finished exactly once (none lost in the pool, none run twice), every thread terminates,
// and the pool never overflows. Run under -fsanitize=thread by tests/test_merge_sim.py for the memory ordering.
//
// usage: merge_sim <waves> <series> <threshold> <seed> [pool entries, default 24576]
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

namespace {

constexpr int SPW = 104;             // slots per wave (C2)
constexpr int kRoom = 64;            // claims fill a wave up to 64 live slots

struct Entry {
    int64_t sid;
    int passes_left;
};

struct Shared {
    std::atomic<uint64_t> work{0};   // ctl[0]
    std::atomic<uint64_t> w40{0};    // ctl[40]
    std::atomic<uint64_t> head{0};   // ctl[41]
    std::atomic<uint64_t> donors{0}; // ctl[42]
    std::vector<Entry> pool;
    std::vector<std::atomic<uint32_t>> ready;
    std::vector<std::atomic<int>> finished;   // per series: times finished
    int64_t N = 0;
    int T = 16;
    uint64_t cap;                    // pool entries (the device: 24 576, the ring's upper three quarters)
    Shared(int64_t n, uint64_t c) : pool(c), ready(c), finished(n), N(n), cap(c) {
        for (auto &r : ready) r.store(0);
        for (auto &f : finished) f.store(0);
    }
};

void wave(Shared &S, int id, uint64_t seed) {
    std::mt19937_64 rng(seed * 7919 + id);
    std::vector<Entry> slot(SPW, Entry{-1, 0});
    S.w40.fetch_add(1);                                  // counted before taking any series
    bool drained = false;
    uint64_t merge_head = 0;
    auto refill = [&](int i) {
        const uint64_t sid = S.work.fetch_add(1);
        if ((int64_t)sid >= S.N) {
            drained = true;
            slot[i].sid = -1;
        } else {
            slot[i].sid = (int64_t)sid;
            slot[i].passes_left = 1 + (int)(rng() % 64) + ((rng() % 97) == 0 ? 2000 : 0);   // a few long ones
        }
    };
    for (int i = 0; i < SPW; ++i) refill(i);
    for (int iter = 0;; ++iter) {
        int live = 0, occ = 0;
        for (auto &e : slot) {
            live += e.sid >= 0;
            occ += e.sid >= 0;
        }
        if (drained) {
            int act = 0;
            uint64_t mbase = 0, mcnt = 0;
            uint64_t w = S.w40.load();
            bool offer = live > 0 && live <= S.T;
            for (;;) {
                const uint64_t active = w & 0xffffffull, tail = w >> 24;
                if (offer) {
                    if (active > 1 && tail + (uint64_t)live <= S.cap) {
                        const uint64_t nw = ((tail + (uint64_t)live) << 24) | (active - 1);
                        if (S.w40.compare_exchange_strong(w, nw)) {
                            act = 1;
                            mbase = tail;
                            break;
                        }
                        continue;                              // w holds the value found
                    }
                    offer = false;
                }
                if (occ < kRoom && tail > merge_head) {
                    uint64_t head = S.head.load();
                    while (head < tail) {
                        const uint64_t c = std::min<uint64_t>(tail - head, (uint64_t)(kRoom - occ));
                        if (S.head.compare_exchange_strong(head, head + c)) {
                            act = 2;
                            mbase = head;
                            mcnt = c;
                            break;
                        }
                    }
                    merge_head = act == 2 ? mbase + mcnt : head;
                    if (act == 2) break;
                }
                if (live > 0) break;
                if (S.w40.compare_exchange_strong(w, w - 1)) {   // leave: every reserved entry claimed
                    act = 3;
                    break;
                }
            }
            if (act == 1) {                                  // hand every live slot over, in slot order
                uint64_t e = mbase;
                for (auto &s : slot)
                    if (s.sid >= 0) {
                        S.pool[e] = s;
                        s.sid = -1;
                        ++e;
                    }
                for (uint64_t k = mbase; k < e; ++k) S.ready[k].store((uint32_t)(k + 1), std::memory_order_release);
                S.donors.fetch_add(1);
                return;
            }
            if (act == 3) return;
            if (act == 2) {                                  // claimed entries into free slots, in order
                uint64_t k = mbase;
                for (auto &s : slot) {
                    if (k == mbase + mcnt) break;
                    if (s.sid < 0) {
                        while (S.ready[k].load(std::memory_order_acquire) != (uint32_t)(k + 1)) std::this_thread::yield();
                        s = S.pool[k];
                        ++k;
                    }
                }
                if (k != mbase + mcnt) {
                    std::fprintf(stderr, "wave %d: claimed %llu entries without room\n", id, (unsigned long long)mcnt);
                    std::abort();
                }
                continue;
            }
        }
        if (live == 0) {                                     // (merge off or an invariant broken: never here)
            std::fprintf(stderr, "wave %d left without the merge protocol\n", id);
            std::abort();
        }
        // one "pass": up to 64 live slots advance; finished ones are written out and refilled
        int served = 0;
        for (int i = 0; i < SPW && served < 64; ++i) {
            Entry &s = slot[(i + iter * 37) % SPW];
            if (s.sid < 0) continue;
            ++served;
            if (--s.passes_left == 0) {
                S.finished[s.sid].fetch_add(1);
                refill((int)(&s - slot.data()));
            }
        }
        if ((rng() & 7) == 0) std::this_thread::yield();
    }
}

}  // namespace

int main(int argc, char **argv) {
    const int W = argc > 1 ? std::atoi(argv[1]) : 64;
    const int64_t N = argc > 2 ? std::atoll(argv[2]) : 50000;
    const int T = argc > 3 ? std::atoi(argv[3]) : 16;
    const uint64_t seed = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 1;
    const uint64_t cap = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 24576;
    Shared S(N, cap);
    S.T = T;
    std::vector<std::thread> th;
    for (int i = 0; i < W; ++i) th.emplace_back(wave, std::ref(S), i, seed);
    for (auto &t : th) t.join();
    int64_t lost = 0, dup = 0;
    for (int64_t i = 0; i < N; ++i) {
        const int f = S.finished[i].load();
        lost += f == 0;
        dup += f > 1;
    }
    const uint64_t w = S.w40.load();
    std::printf("waves %d series %lld threshold %d: handed over %llu series by %llu waves, claimed %llu, active left "
                "%llu, lost %lld, finished twice %lld\n",
                W, (long long)N, T, (unsigned long long)(w >> 24), (unsigned long long)S.donors.load(),
                (unsigned long long)S.head.load(), (unsigned long long)(w & 0xffffff), (long long)lost, (long long)dup);
    return (lost == 0 && dup == 0 && (w >> 24) == S.head.load() && (w & 0xffffff) == 0) ? 0 : 1;
}
