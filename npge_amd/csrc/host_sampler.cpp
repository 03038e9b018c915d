// host_sampler.cpp -- diagnostic sampling profiler of the library's host code
// (no perf on the GPU boxes).  SIGPROF every 1/hz s of process CPU time; the
// handler records the interrupted instruction pointer; npgx_diag_prof_stop
// writes "offset-in-this-library count" lines (symbolize with nm -C).
// Not part of the C ABI header: tools/host_profile.py drives it via ctypes.
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>

namespace {
constexpr int kMax = 1 << 20;
uintptr_t g_pc[kMax];
uintptr_t g_ret[kMax];  // the word at the stack pointer (a leaf's return address)
std::atomic<int> g_n{0};
// call stacks of the first kStk samples (unwound with backtrace(); attributes
// time spent in the HIP runtime / libc to the library function calling it)
constexpr int kStk = 1 << 16, kDepth = 24;
void* g_stk[kStk][kDepth];
int g_stk_n[kStk];

void on_prof(int, siginfo_t*, void* uc) {
    const int i = g_n.fetch_add(1, std::memory_order_relaxed);
    if (i < kMax) {
        const greg_t* g = ((ucontext_t*)uc)->uc_mcontext.gregs;
        g_pc[i] = (uintptr_t)g[REG_RIP];
        g_ret[i] = *(const uintptr_t*)g[REG_RSP];
    }
    if (i < kStk) g_stk_n[i] = backtrace(g_stk[i], kDepth);
}
}  // namespace

extern "C" int npgx_diag_prof_start(int hz) {
    g_n = 0;
    void* warm[4];
    backtrace(warm, 4);  // loads the unwinder outside the signal handler
    struct sigaction sa {};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGPROF, &sa, nullptr) != 0) return -1;
    struct itimerval it {};
    it.it_interval.tv_usec = 1000000 / (hz > 0 ? hz : 1000);
    it.it_value = it.it_interval;
    return setitimer(ITIMER_PROF, &it, nullptr);
}

extern "C" int npgx_diag_prof_stop(const char* path) {
    struct itimerval it {};
    setitimer(ITIMER_PROF, &it, nullptr);
    signal(SIGPROF, SIG_IGN);
    Dl_info self;
    if (!dladdr((void*)&npgx_diag_prof_start, &self)) return -1;
    const uintptr_t base = (uintptr_t)self.dli_fbase;
    std::map<uintptr_t, int> in_lib;
    std::map<std::string, int> other;
    const int n = g_n < kMax ? (int)g_n : kMax;
    for (int i = 0; i < n; i++) {
        Dl_info d;
        if (dladdr((void*)g_pc[i], &d) && d.dli_fbase == self.dli_fbase) in_lib[g_pc[i] - base]++;
        else if (dladdr((void*)g_pc[i], &d) && d.dli_fname) {
            std::string k = std::string(d.dli_fname) + ":" + (d.dli_sname ? d.dli_sname : "?");
            Dl_info c;
            if (d.dli_sname && std::string(d.dli_sname) == "ioctl" && dladdr((void*)g_ret[i], &c) && c.dli_fname)
                k += std::string("<-") + c.dli_fname + ":" + (c.dli_sname ? c.dli_sname : "?");
            other[k]++;
        }
        else
            other["?"]++;
    }
    // samples outside the library: the innermost library frames on the stack
    std::map<std::pair<uintptr_t, uintptr_t>, int> callers;
    for (int i = 0; i < std::min(n, kStk); i++) {
        Dl_info d;
        if (dladdr((void*)g_pc[i], &d) && d.dli_fbase == self.dli_fbase) continue;
        uintptr_t c0 = 0, c1 = 0;
        for (int k = 0; k < g_stk_n[i]; k++) {
            Dl_info e;
            if (!dladdr(g_stk[i][k], &e) || e.dli_fbase != self.dli_fbase) continue;
            const uintptr_t off = (uintptr_t)g_stk[i][k] - base;
            if (!c0) c0 = off;
            else if (!c1) { c1 = off; break; }
        }
        callers[{c0, c1}]++;  // (0, 0): no library frame (another thread)
    }
    FILE* f = fopen(path, "w");
    if (!f) return -1;
    fprintf(f, "# samples %d\n", n);
    for (auto& kv : callers) fprintf(f, "caller %lx %lx %d\n", (unsigned long)kv.first.first,
                                     (unsigned long)kv.first.second, kv.second);
    for (auto& kv : other) fprintf(f, "lib %s %d\n", kv.first.c_str(), kv.second);
    for (auto& kv : in_lib) fprintf(f, "%lx %d\n", (unsigned long)kv.first, kv.second);
    fclose(f);
    return 0;
}
