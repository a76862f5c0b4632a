// at2v_pack.h — record packer: SendAssetRequest wire fields -> verify records.
//
// Reference: the client builds SendAssetRequest{sender = bincode(A), sequence, recipient = bincode(B),
// amount, signature = bincode(R||S)} (/root/reference/src/client.rs:77-88, src/at2.proto:10-16) and
// signs M = bincode(ThinTransaction{recipient, amount}) (src/lib.rs:14-22, client.rs:77-78). The server
// decodes recipient (rpc.rs:265), sender (:269) and signature (:281) with bincode, failing the RPC
// with InvalidArgument on the first error, in that order.
//
// Wire encodings of drop's PublicKey/Signature (crate not in the tree, SURVEY a1: UNVERIFIED):
//   WIRE_BYTES : serde bytes  -> bincode u64le(len) || bytes   (40 B key, 72 B signature; default)
//   WIRE_ARRAY : fixed array  -> raw bytes, no prefix           (32 B key, 64 B signature)
// bincode's legacy `deserialize` accepts trailing bytes, so only the prefix and the minimum size are
// checked here. Whether the key bytes are a valid curve point is the GPU's job (at2v_decode_points for
// the recipient; the verify kernel's V2 for the sender).
#pragma once
#include <cstdint>
#include <cstring>

namespace at2v {

enum WireEncoding : int { kWireBytes = 0, kWireArray = 1 };
enum PackStatus : uint8_t { kPackOk = 0, kPackBadRecipient = 1, kPackBadSender = 2, kPackBadSignature = 3 };

inline uint64_t load_u64le(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}
inline void store_u64le(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

// bincode field of `len` bytes: returns a pointer to the payload or nullptr on a framing error
inline const uint8_t* wire_field(const uint8_t* p, size_t n, size_t len, int enc) {
  if (!p) return nullptr;
  if (enc == kWireArray) return n >= len ? p : nullptr;
  if (n < 8 + len || load_u64le(p) != len) return nullptr;
  return p + 8;
}

// bytes of bincode(ThinTransaction{recipient, amount}) for the given key encoding
inline size_t thin_transaction_len(int enc) { return (enc == kWireArray ? 32 : 40) + 8; }

inline size_t thin_transaction(uint8_t* out, const uint8_t recipient[32], uint64_t amount, int enc) {
  size_t o = 0;
  if (enc == kWireBytes) {
    store_u64le(out, 32);
    o = 8;
  }
  std::memcpy(out + o, recipient, 32);
  store_u64le(out + o + 32, amount);
  return o + 40;
}

}  // namespace at2v
