#include "tunnel/session.h"

namespace p2pt {

std::shared_ptr<void> connect_webrtc(Reactor& r, const AppConfig&, ConnectCb cb) {
  r.post([cb] { cb(nullptr, "webrtc transport not available yet"); });
  return nullptr;
}

}  // namespace p2pt
