"""CPU: the apply step (at2v_ledger_*, host C++ in libat2v.so) against the reference's own tests and the
behaviour of its deliver/apply loop. No GPU: the ledger consumes verdict bitmaps, it does not verify.

Mirrored reference tests (/root/reference):
  accounts/account.rs:57-90     debit_too_much_fails, debit_increase_sequence, credit_doesnt_change_sequence
  accounts/mod.rs:216-300       new_account_is_the_same_as_unknown_account,
                                transfer_to_themselves_increment_sequence_and_keep_balance,
                                transfer_too_much_fails_and_increases_sequence
  recent_transactions.rs:203-248 put_transactions_show_in_get_all
  tests/send-asset-to-itself-keep-balance, tests/send-two-tx-with-same-content-works,
  tests/sent-tx-shows-in-latest-txs   (end-to-end CLI scenarios, replayed at the ledger boundary)
"""
import numpy as np
import pytest

from at2v.node import (INITIAL_BALANCE, TX_FAILURE, TX_INCONSECUTIVE_SEQUENCE, TX_PENDING, TX_SUCCESS, TX_UNDERFLOW,
                       AccountError, Ledger)


def key(i: int) -> bytes:
    return bytes([i]) * 32


A, B, C = key(1), key(2), key(3)


@pytest.fixture
def led():
    l = Ledger()
    yield l
    l.close()


def deliver(led, txs, verdicts=None, now_us=0):
    """txs = [(sender, seq, recipient, amount)]"""
    n = len(txs)
    snd = np.frombuffer(b"".join(t[0] for t in txs), np.uint8).reshape(n, 32)
    rcp = np.frombuffer(b"".join(t[2] for t in txs), np.uint8).reshape(n, 32)
    return led.deliver(snd, np.array([t[1] for t in txs], np.uint32), rcp, np.array([t[3] for t in txs], np.uint64),
                       verdicts, now_us)


# ---- account.rs tests
def test_debit_too_much_fails(led):
    with pytest.raises(AccountError) as e:
        led.transfer(A, 1, B, INITIAL_BALANCE + 1)
    assert e.value.code == TX_UNDERFLOW
    assert led.last_sequence(A) == 1  # sequence consumed although the debit failed
    assert led.balance(A) == INITIAL_BALANCE


def test_debit_increase_sequence(led):
    led.transfer(A, 1, B, 1)
    assert led.last_sequence(A) == 1


def test_credit_doesnt_change_sequence(led):
    led.transfer(A, 1, B, 1)
    assert led.last_sequence(B) == 0 and led.balance(B) == INITIAL_BALANCE + 1


# ---- accounts/mod.rs tests
def test_new_account_is_the_same_as_unknown_account(led):
    assert led.balance(key(9)) == INITIAL_BALANCE and led.last_sequence(key(9)) == 0


def test_transfer_to_themselves_increment_sequence_and_keep_balance(led):
    led.transfer(A, 1, A, 10)
    assert led.balance(A) == INITIAL_BALANCE and led.last_sequence(A) == 1


def test_transfer_too_much_fails_and_increases_sequence(led):
    with pytest.raises(AccountError):
        led.transfer(A, 1, B, INITIAL_BALANCE + 1)
    assert led.balance(A) == INITIAL_BALANCE and led.last_sequence(A) == 1
    assert led.balance(B) == INITIAL_BALANCE and led.last_sequence(B) == 0


def test_inconsecutive_sequence_changes_nothing(led):
    with pytest.raises(AccountError) as e:
        led.transfer(A, 2, B, 5)
    assert e.value.code == TX_INCONSECUTIVE_SEQUENCE
    assert led.last_sequence(A) == 0 and led.balance(A) == INITIAL_BALANCE and led.balance(B) == INITIAL_BALANCE


def test_huge_amount_underflows_before_any_credit(led):
    """the receiver's checked_add (Overflow) is unreachable from INITIAL_BALANCE accounts: the sender's
    debit fails first (Underflow), consuming the sequence and leaving the receiver untouched"""
    with pytest.raises(AccountError) as e:
        led.transfer(A, 1, B, 2**64 - 1)
    assert e.value.code == TX_UNDERFLOW and led.last_sequence(A) == 1 and led.balance(B) == INITIAL_BALANCE


# ---- recent_transactions.rs tests
def test_put_transactions_show_in_get_all(led):
    led.recent_put(A, 1, B, 10)
    led.recent_put(A, 2, A, 3)
    got = led.recent()
    assert [(t.sender, t.sender_sequence, t.recipient, t.amount, t.state) for t in got] == [
        (A, 1, B, 10, TX_PENDING), (A, 2, A, 3, TX_PENDING)]


def test_recent_is_a_10_entry_fifo_and_put_is_idempotent(led):
    for s in range(1, 13):
        led.recent_put(A, s, B, s)
    led.recent_put(A, 12, B, 999)  # NOP: (sender, sequence) already present
    got = led.recent()
    assert [t.sender_sequence for t in got] == list(range(3, 13))
    assert got[-1].amount == 12


# ---- Service::spawn deliver/apply loop (rpc.rs:149-211)
def test_verified_payload_is_applied_and_marked_success(led):
    led.recent_put(A, 1, B, 10)
    st = deliver(led, [(A, 1, B, 10)])
    assert st["applied"] == 1 and st["requeued"] == 0
    assert led.balance(A) == INITIAL_BALANCE - 10 and led.balance(B) == INITIAL_BALANCE + 10
    assert led.recent()[0].state == TX_SUCCESS


def test_rejected_verdicts_are_never_applied(led):
    st = deliver(led, [(A, 1, B, 10), (C, 1, B, 7)], verdicts=np.array([False, True]))
    assert st["rejected"] == 1 and st["delivered"] == 1 and st["applied"] == 1
    assert led.balance(A) == INITIAL_BALANCE and led.last_sequence(A) == 0
    assert led.balance(B) == INITIAL_BALANCE + 7


def test_failed_batch_verdicts_apply_nothing(led):
    """the queue reports 0xff for every record of a batch that failed on the device. Such
    verdicts must never read as valid: delivery raises before anything reaches the ledger."""
    from at2v.node import BatchFailedError
    txs = [(A, 1, B, 10), (C, 1, B, 7), (A, 2, B, 1)]
    for bad in (np.array([0xFF, 0xFF, 0xFF], np.uint8), np.array([1, 0xFF, 1], np.uint8)):
        with pytest.raises(BatchFailedError):
            deliver(led, txs, verdicts=bad)
    for bad in (np.array([1, 2, 1], np.uint8), np.array([1, 0], np.uint8), np.array([0.0, 1.0, 1.0])):
        with pytest.raises(ValueError):
            deliver(led, txs, verdicts=bad)
    assert led.pending() == 0 and led.balance(A) == INITIAL_BALANCE and led.balance(B) == INITIAL_BALANCE
    assert led.last_sequence(A) == 0 and led.last_sequence(C) == 0
    # plain 0/1 integers (queue bytes, Python lists) are per-record verdicts, never bitmap words
    st = deliver(led, txs, verdicts=[0, 1, 0])
    assert st["delivered"] == 1 and st["rejected"] == 2 and led.balance(B) == INITIAL_BALANCE + 7


def test_bitmap_words_select_records(led):
    n = 40
    snd = np.repeat(np.frombuffer(C, np.uint8)[None], n, 0)
    rcp = np.repeat(np.frombuffer(B, np.uint8)[None], n, 0)
    words = np.array([0b101, 1 << 7], np.uint32)  # records 0, 2 and 39
    st = led.deliver(snd, np.arange(1, n + 1, dtype=np.uint32), rcp, np.ones(n, np.uint64), words=words)
    assert st["delivered"] == 3 and st["rejected"] == n - 3 and st["applied"] == 1  # seq 1 only: 3 and 40 wait
    with pytest.raises(ValueError):
        led.deliver(snd, np.arange(1, n + 1, dtype=np.uint32), rcp, np.ones(n, np.uint64),
                    words=np.array([5, 0, 0], np.uint32))


def test_out_of_order_sequences_apply_over_several_passes(led):
    """into_sorted_vec of BinaryHeap<Reverse<_>> walks the payloads in DESCENDING order: seq 3, 2, 1 take
    three passes to apply, and the loop stops after a pass that does not shrink the set"""
    st = deliver(led, [(A, 1, B, 1), (A, 3, B, 3), (A, 2, B, 2)])
    assert st["applied"] == 3 and st["requeued"] == 0 and st["passes"] == 4
    assert led.last_sequence(A) == 3 and led.balance(B) == INITIAL_BALANCE + 6


def test_gap_stays_pending_until_filled(led):
    st = deliver(led, [(A, 2, B, 2)])
    assert st["applied"] == 0 and st["requeued"] == 1 and led.pending() == 1
    st = deliver(led, [(A, 1, B, 1)])
    assert st["applied"] == 2 and led.pending() == 0 and led.last_sequence(A) == 2


def test_underflow_consumes_the_sequence_and_is_retried_forever(led):
    led.recent_put(A, 1, B, INITIAL_BALANCE + 1)
    st = deliver(led, [(A, 1, B, INITIAL_BALANCE + 1)])
    assert st["applied"] == 0 and st["requeued"] == 1
    assert led.last_sequence(A) == 1 and led.balance(A) == INITIAL_BALANCE
    assert led.recent()[0].state == TX_PENDING
    # the next transaction of A (sequence 2) goes through; the failed one stays pending
    st = deliver(led, [(A, 2, B, 5)])
    assert st["applied"] == 1 and led.pending() == 1 and led.balance(B) == INITIAL_BALANCE + 5


def test_ttl_expiry_marks_failure_but_still_processes(led):
    """rpc.rs:183-195: no `continue` after the TTL branch"""
    led.recent_put(A, 2, B, 5)
    deliver(led, [(A, 2, B, 5)], now_us=0)  # gap: pending
    assert led.recent()[0].state == TX_PENDING
    st = deliver(led, [(C, 1, B, 1)], now_us=61_000_000)  # 61 s later: expired, still fails (gap)
    assert st["expired"] >= 1 and led.recent()[0].state == TX_FAILURE
    st = deliver(led, [(A, 1, B, 1)], now_us=62_000_000)  # gap filled: the expired one applies after all
    assert led.last_sequence(A) == 2 and led.recent()[0].state == TX_SUCCESS


def test_cli_send_asset_to_itself_keep_balance(led):
    """tests/send-asset-to-itself-keep-balance"""
    deliver(led, [(A, 1, A, 10)])
    assert led.balance(A) == INITIAL_BALANCE and led.last_sequence(A) == 1


def test_cli_send_two_tx_with_same_content_works(led):
    """tests/send-two-tx-with-same-content-works: same (recipient, amount) at sequences 1 and 2"""
    for s in (1, 2):
        led.recent_put(A, s, B, 5)
    deliver(led, [(A, 1, B, 5)])
    deliver(led, [(A, 2, B, 5)])
    txs = led.recent()
    assert len(txs) == 2 and all(t.sender == A and t.recipient == B and t.amount == 5 for t in txs)
    assert all(t.state == TX_SUCCESS for t in txs)


def test_cli_sent_tx_shows_in_latest_txs(led):
    led.recent_put(A, 1, B, 10)
    deliver(led, [(A, 1, B, 10)])
    (t,) = led.recent()
    assert (t.sender, t.recipient, t.amount, t.state) == (A, B, 10, TX_SUCCESS)


def test_order_dependent_balances_match_python_restatement(led):
    """random multi-sender traffic with gaps, reorderings and overdrafts, against a direct Python restatement
    of rpc.rs:149-211 + accounts/*.rs (the same algorithm written independently here)"""
    rng = np.random.default_rng(5)
    keys = [key(i) for i in range(1, 7)]
    seqs = {k: 0 for k in keys}
    batches = []
    for _ in range(12):
        b = []
        for _ in range(rng.integers(1, 25)):
            s = keys[rng.integers(len(keys))]
            seqs[s] += 1
            seq = seqs[s] if rng.random() > 0.1 else seqs[s] + 3  # some gaps
            r = keys[rng.integers(len(keys))]
            amt = int(rng.integers(1, 60000))
            b.append((s, seq, r, amt))
        rng.shuffle(b)
        batches.append(b)

    # python restatement
    acct = {}

    def get(k):
        return acct.get(k, [0, INITIAL_BALANCE])

    def transfer(s, q, r, amt):
        if s == r:
            a = acct.setdefault(s, [0, INITIAL_BALANCE])
            if a[0] + 1 != q:
                return 1
            a[0] = q
            return 0
        sa, ra = list(get(s)), list(get(r))
        if sa[0] + 1 != q:
            acct[s] = sa
            return 1
        sa[0] = q
        if sa[1] < amt:
            acct[s] = sa
            return 3
        sa[1] -= amt
        acct[s] = sa
        if ra[1] + amt >= 2**64:
            return 2
        ra[1] += amt
        acct[r] = ra
        return 0

    pending = []
    arrival = 0
    for b in batches:
        for t in b:
            pending.append((t[1], t[0], t[2], t[3], 0, arrival))
            arrival += 1
        prev = None
        while prev is None or len(pending) < prev:
            prev = len(pending)
            rem = []
            for p in sorted(pending, reverse=True):
                if transfer(p[1], p[0], p[2], p[3]):
                    rem.append(p)
            pending = rem
        deliver(led, b)
    for k in keys:
        assert led.balance(k) == get(k)[1], k
        assert led.last_sequence(k) == get(k)[0], k
    assert led.pending() == len(pending)
