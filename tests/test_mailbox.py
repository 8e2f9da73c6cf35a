"""CPU side of the HBM mailboxes: the SeqFold audit and the mailbox Send reference.

The audit is what the GPU tests (test_mailbox_gpu.py) rely on to prove
exactly-once, serialised, FIFO execution, so it must itself reject every
kind of violation: a lost message, a duplicated one, a lost update (two
messages that saw the same state), and a wrong final state.
"""
import numpy as np
import torch

from ptype_amd.ops import batch as B
from ptype_amd.ops.mailbox import audit_fold, batch_ordered, send_ref
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_SEQ_FOLD, STATUS_NO_ACTOR, method_ordered


def serial_run(mbox, a0, state0, order):
    state = state0.clone()
    reply = torch.zeros(len(mbox), dtype=torch.int64)
    for i in order:
        x = int(mbox[i])
        reply[i] = state[x]
        state[x] = B.fold_step(int(state[x]), int(a0[i]))
    return reply, state


def test_audit_accepts_any_serial_order_and_recovers_it():
    g = torch.Generator().manual_seed(0)
    n, M = 16, 400
    mbox = torch.randint(0, n, (M,), generator=g)
    a0 = torch.randint(-(1 << 40), 1 << 40, (M,), generator=g)
    s0 = torch.randint(0, 1 << 30, (n,), generator=g)
    order = torch.randperm(M, generator=g).tolist()
    reply, s1 = serial_run(mbox, a0, s0, order)
    ok, got = audit_fold(mbox, a0, reply, np.zeros(M, dtype=np.int32), s0, s1)
    assert ok, got
    for x, seq in got.items():  # the recovered per-actor order is the one that ran
        assert seq == [i for i in order if int(mbox[i]) == x]


def test_audit_rejects_lost_duplicate_and_racy_executions():
    g = torch.Generator().manual_seed(1)
    n, M = 8, 200
    mbox = torch.randint(0, n, (M,), generator=g)
    a0 = torch.randint(1, 1 << 40, (M,), generator=g)
    s0 = torch.zeros(n, dtype=torch.int64)
    order = list(range(M))
    reply, s1 = serial_run(mbox, a0, s0, order)
    st = np.zeros(M, dtype=np.int32)
    # lost message: ran nowhere, but the final state claims the whole chain
    lost, _ = serial_run(mbox, a0, s0, order[:-1])
    ok, why = audit_fold(mbox, a0, lost, st, s0, s1)
    assert not ok
    # duplicated message: applied twice
    twice = order + [order[-1]]
    _, s_dup = serial_run(mbox, a0, s0, twice)
    ok, why = audit_fold(mbox, a0, reply, st, s0, s_dup)
    assert not ok and "chain ends" in why
    # lost update: two messages of one actor read the same state (a racy read-modify-write)
    x = int(mbox[0])
    j = [i for i in order if int(mbox[i]) == x][1]
    racy = reply.clone()
    racy[j] = racy[0]
    ok, why = audit_fold(mbox, a0, racy, st, s0, s1)
    assert not ok
    # any non-OK status fails the audit
    bad = st.copy()
    bad[3] = STATUS_NO_ACTOR
    assert not audit_fold(mbox, a0, reply, bad, s0, s1)[0]


def test_send_ref_runs_in_message_order():
    n, M = 8, 64
    g = torch.Generator().manual_seed(2)
    actor = torch.randint(0, n, (M,), generator=g, dtype=torch.int32)
    a0 = torch.randint(0, 100, (M,), generator=g)
    rank = torch.zeros(M, dtype=torch.int32)
    rank[5] = 1  # one message for another rank: no actor here
    mbox = actor.long() ^ 3
    state = torch.arange(n, dtype=torch.int64)
    s0 = state.clone()
    v, st = send_ref(B.MsgBatch(actor, a0, None, None, METHOD_SEQ_FOLD), rank, mbox, state)
    assert int(st[5]) == STATUS_NO_ACTOR
    keep = torch.ones(M, dtype=torch.bool)
    keep[5] = False
    ok, order = audit_fold(mbox[keep], a0[keep], v[keep], st[keep].numpy(), s0, state)
    assert ok, order
    for seq in order.values():
        assert seq == sorted(seq)  # message order


def test_ordered_method_classification():
    assert method_ordered(METHOD_SEQ_FOLD) and not method_ordered(METHOD_CALC_MULTIPLY)
    assert batch_ordered(B.MsgBatch(torch.zeros(1, dtype=torch.int32), torch.zeros(1), None, None, METHOD_SEQ_FOLD))
    assert not batch_ordered(B.MsgBatch(torch.zeros(1, dtype=torch.int32), torch.zeros(1), None, None, 1))
    # a method column may carry an ordered method
    assert batch_ordered(B.MsgBatch(torch.zeros(1, dtype=torch.int32), torch.zeros(1), None, None,
                                    torch.ones(1, dtype=torch.int16)))
