// WebRTC session establishment: signalling, role election, offer/answer FSMs.
//
// Mirrors reference tunnel/src/rtc.rs:
//   - connect(): join room; if `peers` is empty wait for peer-joined and be
//     the OFFERER, else be the ANSWERER                          (:463-514)
//   - offerer: create DC "tunnel", offer, wait <= 5 s for gathering, send the
//     full SDP; apply answer; apply/buffer trickled candidates     (:126-273)
//   - answerer: on offer set remote, flush buffered candidates, answer after
//     <= 5 s gathering; take the remote-created DC                  (:276-460)
//   - peer-left / signalling error / EOF / ICE failure -> error     (:224-232, :408-416)
// Fix vs. reference (Q7): a stray message while waiting for peer-joined no
// longer drops the first peer back into the "wait for joined" loop.
#pragma once

#include <memory>

#include "rtc/peer.h"
#include "tunnel/app.h"

namespace p2pt {

std::shared_ptr<void> connect_webrtc(Reactor& r, const AppConfig& cfg, ConnectCb cb);
// The PeerConnection configuration a role's connections use (the first one
// and the "assoc" extension's extra ones).
rtc::PcConfig make_pc_config(const AppConfig& cfg);

}  // namespace p2pt
