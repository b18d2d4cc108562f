// copy_probe.hip -- what a chunked pinned H2D pipeline costs on this box,
// in host wall time per call (median of N calls per variant, rotated):
// the a14 log (75.5 MB by default) copied
//   single      one hipMemcpyAsync on a copy stream, synchronized
//   k<K>        K chunks (weights K..1) back to back, no events
//   k<K>ev      K chunks, an event recorded after each
//   k<K>kern    + the compute stream waits on each event and launches a
//               one-workgroup kernel per chunk (the a14 shape)
//   k<K>kern0   + the copy stream first waits on an event of the (idle)
//               compute stream (what every a14 call does today)
//   single+k    one copy, then one kernel on the SAME stream
//   *-spin      the host polls hipStreamQuery instead of hipStreamSynchronize
//   small       a 4 KiB copy: the fixed round trip of one copy and its wait
//   k<K>kernnf  k<K>kern with hipEventDisableSystemFence events
//   k<K>wv      chunk flags by hipStreamWriteValue32 on the copy stream,
//               the compute stream waits by hipStreamWaitValue32
// Diagnosis only; nothing on the product path uses it.
//
// usage: copy_probe [MB=75.5] [calls=100]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void k_touch(const uint8_t *p, uint64_t n, uint32_t *out) {
    // reads one byte per 4 KiB page of its chunk: a stand-in for a group kernel
    uint32_t x = 0;
    for (uint64_t i = threadIdx.x * 4096ull; i < n; i += 4096ull * blockDim.x) x += p[i];
    if (x == 0xdeadbeef) out[0] = x;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const double mb = argc > 1 ? atof(argv[1]) : 75.5;
    const int calls = argc > 2 ? atoi(argv[2]) : 100;
    const uint64_t len = (uint64_t)(mb * 1e6) & ~4095ull;
    uint8_t *h, *d;
    uint32_t *dflag, *dout;
    CK(hipHostMalloc((void **)&h, len, hipHostMallocDefault));
    memset(h, 1, len);
    CK(hipMalloc((void **)&d, len));
    CK(hipMalloc((void **)&dflag, 64 * 4));
    CK(hipMalloc((void **)&dout, 4));
    CK(hipMemset(dflag, 0, 64 * 4));
    hipStream_t cs, ks;
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(17), evn(17);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto &e : evn) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    uint32_t seq = 0;

    auto cuts = [&](int K) {
        std::vector<uint64_t> c(K + 1, 0);
        const uint64_t w = (uint64_t)K * (K + 1) / 2;
        for (int k = 1; k < K; k++) {
            const uint64_t pre = (uint64_t)k * K - (uint64_t)k * (k - 1) / 2;
            c[k] = (uint64_t)((double)len * pre / w) & ~4095ull;
        }
        c[K] = len;
        return c;
    };
    struct V {
        std::string name;
        std::function<void()> run;
    };
    std::vector<V> vs;
    vs.push_back({"single", [&] {
                      CK(hipMemcpyAsync(d, h, len, hipMemcpyHostToDevice, cs));
                      CK(hipStreamSynchronize(cs));
                  }});
    vs.push_back({"single-spin", [&] {  // the same, the host polling the stream
                      CK(hipMemcpyAsync(d, h, len, hipMemcpyHostToDevice, cs));
                      while (hipStreamQuery(cs) == hipErrorNotReady) (void)hipGetLastError();
                  }});
    vs.push_back({"small", [&] {  // 4 KiB: the round trip of one copy + wait
                      CK(hipMemcpyAsync(d, h, 4096, hipMemcpyHostToDevice, cs));
                      CK(hipStreamSynchronize(cs));
                  }});
    vs.push_back({"small-spin", [&] {
                      CK(hipMemcpyAsync(d, h, 4096, hipMemcpyHostToDevice, cs));
                      while (hipStreamQuery(cs) == hipErrorNotReady) (void)hipGetLastError();
                  }});
    vs.push_back({"single+k", [&] {
                      CK(hipMemcpyAsync(d, h, len, hipMemcpyHostToDevice, cs));
                      hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, cs, d, len, dout);
                      CK(hipStreamSynchronize(cs));
                  }});
    // the a14 shape: 5 : 2 : 1 chunks, each kernel behind its chunk's event
    // (k521kern), and the same with the chunk boundaries overlapped on two copy
    // streams (k521ov<T>: chunk j+1 starts on the other stream once chunk j has
    // only its last T MiB left, so the boundary's event and setup run under
    // that tail instead of leaving the link idle)
    hipStream_t cs2;
    CK(hipStreamCreateWithFlags(&cs2, hipStreamNonBlocking));
    std::vector<hipEvent_t> evp(17);
    for (auto &e : evp) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    auto cut521 = [&]() {
        std::vector<uint64_t> c{0, (uint64_t)((double)len * 5 / 8) & ~4095ull,
                                (uint64_t)((double)len * 7 / 8) & ~4095ull, len};
        return c;
    };
    vs.push_back({"k521kern", [&] {
                      auto c = cut521();
                      for (int j = 0; j < 3; j++) {
                          CK(hipMemcpyAsync(d + c[j], h + c[j], c[j + 1] - c[j], hipMemcpyHostToDevice, cs));
                          CK(hipEventRecord(evn[j], cs));
                      }
                      for (int j = 0; j < 3; j++) {
                          CK(hipStreamWaitEvent(ks, evn[j], 0));
                          hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, ks, d + c[j], c[j + 1] - c[j], dout);
                      }
                      CK(hipStreamSynchronize(ks));
                      CK(hipStreamSynchronize(cs));
                  }});
    for (int T : {1, 2, 4})
        vs.push_back({"k521ov" + std::to_string(T), [&, T] {
                          auto c = cut521();
                          const uint64_t tail = (uint64_t)T << 20;
                          for (int j = 0; j < 3; j++) {
                              hipStream_t s = (j & 1) ? cs2 : cs;
                              if (j) CK(hipStreamWaitEvent(s, evp[j - 1], 0));
                              const uint64_t mid = c[j + 1] - std::min(tail, (c[j + 1] - c[j]) / 2);
                              CK(hipMemcpyAsync(d + c[j], h + c[j], mid - c[j], hipMemcpyHostToDevice, s));
                              CK(hipEventRecord(evp[j], s));
                              CK(hipMemcpyAsync(d + mid, h + mid, c[j + 1] - mid, hipMemcpyHostToDevice, s));
                              CK(hipEventRecord(evn[j], s));
                          }
                          for (int j = 0; j < 3; j++) {
                              CK(hipStreamWaitEvent(ks, evn[j], 0));
                              hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, ks, d + c[j], c[j + 1] - c[j], dout);
                          }
                          CK(hipStreamSynchronize(ks));
                          CK(hipStreamSynchronize(cs));
                          CK(hipStreamSynchronize(cs2));
                      }});
    for (int K : {2, 3, 4}) {
        const std::string k = "k" + std::to_string(K);
        vs.push_back({k, [&, K] {
                          auto c = cuts(K);
                          for (int j = 0; j < K; j++)
                              CK(hipMemcpyAsync(d + c[j], h + c[j], c[j + 1] - c[j], hipMemcpyHostToDevice, cs));
                          CK(hipStreamSynchronize(cs));
                      }});
        vs.push_back({k + "ev", [&, K] {
                          auto c = cuts(K);
                          for (int j = 0; j < K; j++) {
                              CK(hipMemcpyAsync(d + c[j], h + c[j], c[j + 1] - c[j], hipMemcpyHostToDevice, cs));
                              CK(hipEventRecord(ev[j], cs));
                          }
                          CK(hipStreamSynchronize(cs));
                      }});
        for (int w0 : {0, 1})
            vs.push_back({k + (w0 ? "kern0" : "kern"), [&, K, w0] {
                              auto c = cuts(K);
                              if (w0) {
                                  CK(hipEventRecord(ev[16], ks));
                                  CK(hipStreamWaitEvent(cs, ev[16], 0));
                              }
                              for (int j = 0; j < K; j++) {
                                  CK(hipMemcpyAsync(d + c[j], h + c[j], c[j + 1] - c[j], hipMemcpyHostToDevice, cs));
                                  CK(hipEventRecord(ev[j], cs));
                              }
                              for (int j = 0; j < K; j++) {
                                  CK(hipStreamWaitEvent(ks, ev[j], 0));
                                  hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, ks, d + c[j], c[j + 1] - c[j], dout);
                              }
                              CK(hipStreamSynchronize(ks));
                              CK(hipStreamSynchronize(cs));
                          }});
        vs.push_back({k + "kernnf", [&, K] {  // k<K>kern with events without the system fence
                          auto c = cuts(K);
                          for (int j = 0; j < K; j++) {
                              CK(hipMemcpyAsync(d + c[j], h + c[j], c[j + 1] - c[j], hipMemcpyHostToDevice, cs));
                              CK(hipEventRecord(evn[j], cs));
                          }
                          for (int j = 0; j < K; j++) {
                              CK(hipStreamWaitEvent(ks, evn[j], 0));
                              hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, ks, d + c[j], c[j + 1] - c[j], dout);
                          }
                          CK(hipStreamSynchronize(ks));
                          CK(hipStreamSynchronize(cs));
                      }});
        vs.push_back({k + "wv", [&, K] {
                          auto c = cuts(K);
                          seq++;
                          for (int j = 0; j < K; j++) {
                              CK(hipMemcpyAsync(d + c[j], h + c[j], c[j + 1] - c[j], hipMemcpyHostToDevice, cs));
                              CK(hipStreamWriteValue32(cs, dflag + j, seq, 0));
                          }
                          for (int j = 0; j < K; j++) {
                              CK(hipStreamWaitValue32(ks, dflag + j, seq, hipStreamWaitValueGte, 0xffffffffu));
                              hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, ks, d + c[j], c[j + 1] - c[j], dout);
                          }
                          CK(hipStreamSynchronize(ks));
                          CK(hipStreamSynchronize(cs));
                      }});
    }
    // warm: clocks and first-touch of every path
    const double t_end = now_us() + 2e6;
    while (now_us() < t_end)
        for (auto &v : vs) v.run();
    std::vector<std::vector<double>> t(vs.size());
    for (int i = 0; i < calls; i++)
        for (size_t j = 0; j < vs.size(); j++) {
            const double a = now_us();
            vs[j].run();
            t[j].push_back(now_us() - a);
        }
    printf("# copy_probe %.1f MB (%llu bytes), %d calls per variant, host wall us (median / min), GB/s at the median\n",
           mb, (unsigned long long)len, calls);
    for (size_t j = 0; j < vs.size(); j++) {
        auto &x = t[j];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        printf("%-10s %8.1f %8.1f  %6.1f\n", vs[j].name.c_str(), med, x[0], len / med / 1e3);
    }
    return 0;
}
