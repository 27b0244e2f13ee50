// `tunnel-signal` — the rendezvous server.
// Arguments as reference signal-server/src/index.ts:82-91: --listen HOST[:PORT]
// (default 0.0.0.0) and --port PORT (default 8787); also reads $PORT like the
// Fly deployment (signal-server/Dockerfile:15).
#include <signal.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "core/log.h"
#include "core/reactor.h"
#include "signal/signal_server.h"

int main(int argc, char** argv) {
  p2pt::log::init_from_env();
  std::string host = "0.0.0.0";
  int port = 8787;
  if (const char* ep = getenv("PORT")) port = atoi(ep);
  bool host_has_port = false;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if ((a == "--listen" || a == "--port") && i + 1 >= argc) {
      fprintf(stderr, "missing value for %s\n", a.c_str());
      return 2;
    }
    if (a == "--listen") {
      host = argv[++i];
    } else if (a == "--port") {
      port = atoi(argv[++i]);
    } else if (a == "-h" || a == "--help") {
      printf("Usage: tunnel-signal [--listen HOST[:PORT]] [--port PORT]\n");
      return 0;
    }
  }
  std::string hostport;
  if (!host.empty() && host[0] == '[') {
    size_t rb = host.find(']');
    host_has_port = rb != std::string::npos && rb + 1 < host.size() && host[rb + 1] == ':';
    hostport = host_has_port ? host : host + ":" + std::to_string(port);
  } else if (host.find(':') != std::string::npos && host.find(':') == host.rfind(':')) {
    hostport = host;  // host:port
  } else {
    hostport = host + ":" + std::to_string(port);
  }
  signal(SIGPIPE, SIG_IGN);
  p2pt::Reactor r;
  p2pt::SignalServer srv(r);
  std::string err;
  if (!srv.listen(hostport, &err)) {
    fprintf(stderr, "[signal] failed to listen: %s\n", err.c_str());
    return 1;
  }
  r.on_signal(SIGINT, [&] { r.stop(); });
  r.on_signal(SIGTERM, [&] { r.stop(); });
  r.run();
  return 0;
}
