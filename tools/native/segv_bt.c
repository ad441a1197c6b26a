/* Host-side diagnostics: on SIGSEGV/SIGABRT print the native call stack
   (backtrace_symbols_fd: library + offset, resolved offline with addr2line)
   to stderr, then re-raise with the default action.  Loaded by the replay
   probe through ctypes; no GPU code. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig) {
  void* pc[64];
  const int n = backtrace(pc, 64);
  const char msg[] = "\n== native backtrace ==\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(pc, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static char alt_stack[1 << 16];

int segv_bt_install(void) {
  void* warm[1];
  backtrace(warm, 1); /* (loads libgcc before any fault) */
  stack_t ss; /* (a stack of its own: a stack overflow still gets its backtrace) */
  memset(&ss, 0, sizeof ss);
  ss.ss_sp = alt_stack;
  ss.ss_size = sizeof alt_stack;
  if (sigaltstack(&ss, 0)) return -1;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_fault;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESETHAND | SA_ONSTACK;
  return sigaction(SIGSEGV, &sa, 0) | sigaction(SIGABRT, &sa, 0) | sigaction(SIGBUS, &sa, 0);
}
