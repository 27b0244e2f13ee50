// AES-GCM record throughput: the vector implementation (core/aesgcm.h) vs
// OpenSSL EVP, seal and open, at the DTLS record sizes the tunnel produces
// (1200 B internet MTU, 16 KiB and 64 KB same-host jumbo packets).
// Prints one JSON line per (size, direction).
#include <openssl/evp.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "core/aesgcm.h"

using namespace p2pt;
using Clock = std::chrono::steady_clock;

int main() {
  uint8_t key[16] = {1, 2, 3}, iv[12] = {4}, aad[13] = {5}, tag[16];
  for (size_t n : {1200, 16384, 65000}) {
    std::vector<uint8_t> buf(n, 7);
    const int iters = int(4e9 / double(n));
    AesGcm g;
    const bool have = g.init(key, 16);
    double own_seal = 0, own_open = 0, own_gather = 0;
    if (have) {
      auto t0 = Clock::now();
      for (int i = 0; i < iters; i++) g.seal(iv, aad, 13, buf.data(), buf.data(), n, tag);
      own_seal = std::chrono::duration<double>(Clock::now() - t0).count();
      g.seal(iv, aad, 13, buf.data(), buf.data(), n, tag);
      std::vector<uint8_t> pt(n);
      bool ok = true;
      t0 = Clock::now();
      for (int i = 0; i < iters; i++) ok &= g.open(iv, aad, 13, buf.data(), pt.data(), n, tag);
      own_open = std::chrono::duration<double>(Clock::now() - t0).count();
      if (!ok) return 1;
      // SCTP-shaped gather list: common header, DATA chunk header, payload.
      std::vector<uint8_t> hdr(28, 1), out(n);
      iovec iov[3] = {{hdr.data(), 12}, {hdr.data() + 12, 16}, {pt.data(), n - 28}};
      t0 = Clock::now();
      for (int i = 0; i < iters; i++) g.seal_gather(iv, aad, 13, iov, 3, out.data(), n, tag);
      own_gather = std::chrono::duration<double>(Clock::now() - t0).count();
    }
    EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(c, EVP_aes_128_gcm(), nullptr, key, nullptr);
    int l;
    auto t0 = Clock::now();
    for (int i = 0; i < iters; i++) {
      EVP_EncryptInit_ex(c, nullptr, nullptr, nullptr, iv);
      EVP_EncryptUpdate(c, nullptr, &l, aad, 13);
      EVP_EncryptUpdate(c, buf.data(), &l, buf.data(), int(n));
      EVP_EncryptFinal_ex(c, buf.data(), &l);
      EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, tag);
    }
    const double evp_seal = std::chrono::duration<double>(Clock::now() - t0).count();
    EVP_CIPHER_CTX_free(c);
    const double bytes = double(iters) * double(n) / 1e9;
    printf("{\"bytes\": %zu, \"vector\": %s, \"own_seal_GBps\": %.2f, \"own_open_GBps\": %.2f, "
           "\"own_seal_gather_GBps\": %.2f, \"evp_seal_GBps\": %.2f}\n",
           n, have ? "true" : "false", have ? bytes / own_seal : 0.0, have ? bytes / own_open : 0.0,
           have ? bytes / own_gather : 0.0, bytes / evp_seal);
  }
}
