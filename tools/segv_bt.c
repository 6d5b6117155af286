/* Debug aid for probes (tools/rccl_pair_probe.py CGX_PAIR_BT=1): a SIGSEGV
 * handler that prints the native backtrace (frames as library+offset) to
 * stderr, then exits.  Loaded with ctypes; never part of the product. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_segv(int sig, siginfo_t *si, void *ctx) {
  (void)ctx;
  void *f[64];
  const int n = backtrace(f, 64);
  const char msg[] = "segv_bt: native backtrace\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(f, n, 2);
  (void)si;
  _exit(128 + sig);
}

__attribute__((constructor)) static void install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, 0);
}
