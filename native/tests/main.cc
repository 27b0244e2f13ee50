#include <signal.h>
#include <sys/prctl.h>

#include <cstring>

#include "core/log.h"
#include "tests/testing.h"

namespace p2pt::testing {
std::vector<Case>& registry() {
  static std::vector<Case> r;
  return r;
}
int g_failures = 0;
static int g_case_failures = 0;
void fail(const char* file, int line, const std::string& msg) {
  g_failures++;
  g_case_failures++;
  fprintf(stderr, "  %s:%d: %s\n", file, line, msg.c_str());
}
}  // namespace p2pt::testing

int main(int argc, char** argv) {
  using namespace p2pt::testing;
  signal(SIGPIPE, SIG_IGN);
  // The SCTP tests emulate links in real time on the test's own loop (packet
  // times down to 0.24 ms, a 1.2 ms drop-tail queue): 1 us timer slack
  // instead of the default 50 us, so the emulation fires when it schedules.
  prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
  p2pt::log::init(getenv("TEST_LOG") ? getenv("TEST_LOG") : "off");
  const char* filter = argc > 1 ? argv[1] : nullptr;
  int ran = 0, failed = 0;
  for (auto& c : registry()) {
    if (filter && !strstr(c.name, filter)) continue;
    g_case_failures = 0;
    c.fn();
    ran++;
    if (g_case_failures) {
      failed++;
      printf("FAIL %s\n", c.name);
    } else {
      printf("ok   %s\n", c.name);
    }
    fflush(stdout);
  }
  printf("%d tests, %d failed\n", ran, failed);
  return failed ? 1 : 0;
}
