// Debug helper: print a native backtrace on SIGSEGV (loaded via ctypes by probe scripts).
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <cstdlib>
static void handler(int sig) {
  void* buf[64];
  int n = backtrace(buf, 64);
  const char msg[] = "\n=== native backtrace ===\n";
  write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(buf, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
extern "C" void sn_install_segv_bt() { signal(SIGSEGV, handler); }
