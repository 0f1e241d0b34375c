/* Native backtrace on SIGSEGV / SIGBUS / SIGABRT for diagnosing host-side crashes inside
 * the HIP runtime (e.g. a segfault in hipStreamEndCapture): load with ctypes and call
 * segv_trace_install(); the handler prints the native frames to stderr, then restores the
 * previous handler and re-raises.
 *   gcc -O1 -g -shared -fPIC tools/segv_trace.c -o tools/libsegv_trace.so -rdynamic */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_old[32];

static void handler(int sig, siginfo_t *info, void *ctx) {
    (void)ctx;
    void *frames[96];
    char msg[128];
    int n = backtrace(frames, 96);
    const char *name = sig == SIGSEGV ? "SIGSEGV" : sig == SIGBUS ? "SIGBUS" : "SIGABRT";
    int len = 0;
    const char *p = "\n=== native backtrace (";
    write(2, p, strlen(p));
    write(2, name, strlen(name));
    /* fault address */
    unsigned long a = (unsigned long)(info ? info->si_addr : 0);
    char hex[32];
    int k = 0;
    do { int d = a & 15; hex[k++] = d < 10 ? '0' + d : 'a' + d - 10; a >>= 4; } while (a && k < 30);
    len = 0;
    msg[len++] = ' '; msg[len++] = 'a'; msg[len++] = 't'; msg[len++] = ' ';
    msg[len++] = '0'; msg[len++] = 'x';
    while (k > 0) msg[len++] = hex[--k];
    msg[len++] = ')'; msg[len++] = '\n';
    write(2, msg, len);
    backtrace_symbols_fd(frames, n, 2);
    p = "=== end native backtrace\n";
    write(2, p, strlen(p));
    sigaction(sig, &g_old[sig], 0);
    raise(sig);
}

int segv_trace_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    int sigs[3] = {SIGSEGV, SIGBUS, SIGABRT};
    for (int i = 0; i < 3; ++i)
        if (sigaction(sigs[i], &sa, &g_old[sigs[i]]) != 0) return -1;
    return 0;
}
