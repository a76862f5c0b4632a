// at2v_ledger.h — the apply step that consumes verify verdicts, host C++.
//
// Restates, record for record, what the reference server does with a delivered (verified) batch:
//   * Account            /root/reference/src/bin/server/accounts/account.rs:11-54
//       INITIAL_BALANCE 100000 (:17); debit bumps last_sequence BEFORE the balance check (:37-43), so
//       an Underflow still consumes the sequence; credit is checked_add (:29-33).
//   * AccountsHandler    accounts/mod.rs:119-214
//       unknown accounts read as Account::new() (:155-163); self-transfer = debit(seq, 0) (:175-182);
//       otherwise the sender copy is written back even when its debit failed (:184-194), the receiver
//       only on success (:196-199).
//   * RecentTransactions recent_transactions.rs:149-200: 10-entry FIFO, put is a NOP for an existing
//       (sender, sequence) (:155-162), update resolves the LAST match (:182-196).
//   * Service::spawn     rpc.rs:149-211: delivered payloads go into a BinaryHeap<Reverse<(payload,
//       Instant)>>; the "dirty" loop re-runs passes over `into_sorted_vec()` (ascending Reverse, i.e.
//       DESCENDING (sequence, sender, recipient, amount, arrival)) while the pending set shrinks; only
//       AccountModification errors are re-queued (:195-205); a TTL-expired payload (60 s) is marked
//       Failure in recent transactions but is still processed in the same pass — there is no
//       `continue` (:183-193) — and a later success overwrites that state.
//   * process_payload    rpc.rs:213-237: transfer, then recent_transactions.update(Success).
// Ordering of sign::PublicKey is taken as lexicographic over its 32 encoded bytes (drop's type; the
// crate is not in the tree).
#pragma once
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <deque>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace at2v {

using Key = std::array<uint8_t, 32>;

struct KeyHash {
  size_t operator()(const Key& k) const {
    uint64_t h;
    std::memcpy(&h, k.data(), 8);  // encodings of distinct keys differ in their low bytes already
    return (size_t)(h ^ (h >> 29));
  }
};

inline Key make_key(const uint8_t* p) {
  Key k;
  std::memcpy(k.data(), p, 32);
  return k;
}

enum AccountError : int { kAccountOk = 0, kInconsecutiveSequence = 1, kOverflow = 2, kUnderflow = 3 };

constexpr uint64_t kInitialBalance = 100000;          // account.rs:17
constexpr uint64_t kTransactionTtlUs = 60ull * 1000000;  // rpc.rs TRANSACTION_TTL (60 s)
constexpr size_t kLatestTransactionsMax = 10;         // recent_transactions.rs:7

struct Account {
  uint32_t last_sequence = 0;  // sieve::Sequence::MIN
  uint64_t balance = kInitialBalance;
  int credit(uint64_t amount) {
    if (balance + amount < balance) return kOverflow;
    balance += amount;
    return kAccountOk;
  }
  int debit(uint32_t sequence, uint64_t amount) {
    if ((uint32_t)(last_sequence + 1) != sequence) return kInconsecutiveSequence;
    last_sequence = sequence;  // consumed even if the balance check below fails
    if (balance < amount) return kUnderflow;
    balance -= amount;
    return kAccountOk;
  }
};

enum TxState : int { kPending = 0, kSuccess = 1, kFailure = 2 };  // at2.proto FullTransaction.State

struct FullTransaction {
  uint64_t timestamp_us;
  Key sender;
  uint32_t sender_sequence;
  Key recipient;
  uint64_t amount;
  int state;
};

struct Payload {  // (sieve::Sequence, sign::PublicKey, ThinTransaction) + arrival time
  uint32_t sequence;
  Key sender;
  Key recipient;
  uint64_t amount;
  uint64_t added_us;
  uint64_t arrival;  // tie-break for equal payloads: arrival order (Instant)
  bool operator<(const Payload& o) const {
    return std::tie(sequence, sender, recipient, amount, added_us, arrival) <
           std::tie(o.sequence, o.sender, o.recipient, o.amount, o.added_us, o.arrival);
  }
};

struct ApplyStats {
  uint64_t applied = 0;       // transfers that succeeded in this call
  uint64_t requeued = 0;      // AccountModification failures left pending after the loop
  uint64_t expired = 0;       // TTL-expired payloads marked Failure (still processed)
  uint64_t passes = 0;        // passes of the reference's "dirty" loop
  uint64_t rejected = 0;      // records whose verdict bit was 0 (never delivered)
};

class Ledger {
 public:
  // ---- AccountsHandler (accounts/mod.rs:155-214)
  uint64_t balance(const Key& k) const {
    auto it = accounts_.find(k);
    return it == accounts_.end() ? kInitialBalance : it->second.balance;
  }
  uint32_t last_sequence(const Key& k) const {
    auto it = accounts_.find(k);
    return it == accounts_.end() ? 0 : it->second.last_sequence;
  }
  int transfer(const Key& sender, uint32_t seq, const Key& receiver, uint64_t amount) {
    if (sender == receiver) {
      Account& a = accounts_.try_emplace(sender).first->second;
      return a.debit(seq, 0);
    }
    Account s = get_or_new(sender), r = get_or_new(receiver);
    const int sres = s.debit(seq, amount);
    accounts_[sender] = s;  // written back before the error is propagated (mod.rs:192-194)
    if (sres) return sres;
    const int rres = r.credit(amount);
    if (rres) return rres;
    accounts_[receiver] = r;
    return kAccountOk;
  }
  size_t num_accounts() const { return accounts_.size(); }

  // ---- RecentTransactions (recent_transactions.rs:149-200)
  void recent_put(const Key& sender, uint32_t seq, const Key& recipient, uint64_t amount, uint64_t now_us) {
    for (const auto& t : recent_)
      if (t.sender_sequence == seq && t.sender == sender) return;
    if (recent_.size() == kLatestTransactionsMax) recent_.pop_front();
    recent_.push_back(FullTransaction{now_us, sender, seq, recipient, amount, kPending});
  }
  void recent_update(const Key& sender, uint32_t seq, int state) {
    for (auto it = recent_.rbegin(); it != recent_.rend(); ++it)
      if (it->sender_sequence == seq && it->sender == sender) {
        it->state = state;
        return;
      }
  }
  const std::deque<FullTransaction>& recent() const { return recent_; }

  // ---- Service::spawn deliver/apply loop (rpc.rs:149-211)
  // One delivered batch: push every payload, then run the dirty loop to a fixed point.
  void deliver(const std::vector<Payload>& batch, uint64_t now_us, ApplyStats* st) {
    for (const auto& p : batch) {
      pending_.push_back(p);
      pending_.back().arrival = arrivals_++;
    }
    size_t previous_len = SIZE_MAX;
    while (pending_.size() < previous_len) {
      previous_len = pending_.size();
      std::vector<Payload> sorted = std::move(pending_);
      std::sort(sorted.begin(), sorted.end(), [](const Payload& a, const Payload& b) { return b < a; });
      pending_.clear();
      if (st) ++st->passes;
      for (const auto& m : sorted) {
        if (now_us > m.added_us && now_us - m.added_us > kTransactionTtlUs) {
          recent_update(m.sender, m.sequence, kFailure);
          if (st) ++st->expired;
        }
        const int err = transfer(m.sender, m.sequence, m.recipient, m.amount);
        if (err) {
          pending_.push_back(m);  // every account::Error is an AccountModification: retried
        } else {
          recent_update(m.sender, m.sequence, kSuccess);
          if (st) ++st->applied;
        }
      }
    }
    if (st) st->requeued = pending_.size();
  }
  size_t pending() const { return pending_.size(); }

 private:
  Account get_or_new(const Key& k) const {
    auto it = accounts_.find(k);
    return it == accounts_.end() ? Account{} : it->second;
  }
  std::unordered_map<Key, Account, KeyHash> accounts_;
  std::deque<FullTransaction> recent_;
  std::vector<Payload> pending_;
  uint64_t arrivals_ = 0;
};

}  // namespace at2v
