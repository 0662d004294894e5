"""emqx_shared_sub's member pick and ack/nack redispatch, host side
(emqx_amd/broker.py SharedSub; apps/emqx/src/emqx_shared_sub.erl:120-134
dispatch/4, :150-194 dispatch_per_qos/dispatch_with_ack, :239-290 pick/do_pick,
:390-397 is_active_sub).  CPU only: the GPU fan-out hands the host (filter,
group) entries; which member gets the message is decided here.  The members a
random or hash strategy picks are parity-unpinned (rand / phash2);
the retry chain and the results are the reference's."""
import pytest

from emqx_amd.broker import STRATEGIES, SharedSub

G, T = b"g", b"s/+"


def test_no_member_is_no_subscribers():
    s = SharedSub("random")
    assert s.dispatch(G, T, [], b"s/1") == (("error", "no_subscribers"), None, [])
    assert s.pick(G, T, []) is None


@pytest.mark.parametrize("strategy", STRATEGIES)
def test_qos0_and_ack_disabled_never_wait_for_an_answer(strategy):
    """dispatch_per_qos/4: QoS 0, or ack disabled, is a plain send: ok."""
    s = SharedSub(strategy, seed=3)
    calls = []

    def respond(m):
        calls.append(m)
        return "nack"

    res, m, failed = s.dispatch(G, T, [1, 2, 3], b"s/1", b"c", qos=0, ack_enabled=True, respond=respond)
    assert res == ("ok", 1) and m in (1, 2, 3) and failed == [] and calls == []
    res, m, failed = s.dispatch(G, T, [1, 2, 3], b"s/1", b"c", qos=1, ack_enabled=False, respond=respond)
    assert res == ("ok", 1) and failed == [] and calls == []


@pytest.mark.parametrize("strategy", STRATEGIES)
def test_a_nack_goes_to_another_member(strategy):
    """A member that nacks (its queue full), is down or times out is skipped
    and the message goes to a member that has not failed it (dispatch/4's
    [SubPid | FailedSubs])."""
    s = SharedSub(strategy, seed=5)
    first = {}

    def respond(m):
        if not first:
            first["m"] = m
            return "nack"
        return "ack"

    res, m, failed = s.dispatch(G, T, [1, 2, 3], b"s/1", b"c", qos=1, ack_enabled=True, respond=respond)
    assert res == ("ok", 1)
    assert failed == [first["m"]] and m != first["m"] and m in (1, 2, 3)


@pytest.mark.parametrize("strategy", STRATEGIES)
@pytest.mark.parametrize("answer", ["nack", "down", "timeout"])
def test_every_member_failing_ends_in_one_retry_send(strategy, answer):
    """do_pick/6: once every member has failed, one is picked from all of them
    and sent without an ack ({retry, Sub}): still {ok, 1}; each member is asked
    once."""
    s = SharedSub(strategy, seed=7)
    asked = []

    def respond(m):
        asked.append(m)
        return answer

    members = [10, 11, 12, 13]
    res, m, failed = s.dispatch(G, T, members, b"s/1", b"c", qos=2, ack_enabled=True, respond=respond)
    assert res == ("ok", 1) and m in members
    assert sorted(failed) == members and sorted(asked) == members   # each asked once, none twice


def test_sticky_keeps_its_member_and_moves_on_failure():
    """pick(sticky, ...): the stored member while it is active (alive, not
    failed for this delivery); otherwise a random pick among the rest, which
    then sticks."""
    s = SharedSub("sticky", seed=1)
    members = [1, 2, 3]
    _, m0, _ = s.dispatch(G, T, members)
    for _ in range(5):
        assert s.dispatch(G, T, members)[1] == m0
    res, m1, failed = s.dispatch(G, T, members, qos=1, ack_enabled=True, respond=lambda m: "nack" if m == m0 else "ack")
    assert res == ("ok", 1) and failed == [m0] and m1 != m0
    assert s.dispatch(G, T, members)[1] == m1   # sticks to the new one
    dead = {m1}
    _, m2, _ = s.dispatch(G, T, members, alive=lambda m: m not in dead)
    assert m2 != m1   # not alive: is_active_sub/2 false


def test_sticky_member_that_left_the_group_but_lives_is_kept():
    """is_active_sub/2 checks liveness and this delivery's failures, not
    membership (emqx_shared_sub.erl:241-245, 390-391): a sticky member that has
    unsubscribed but is alive still gets the group's messages."""
    s = SharedSub("sticky", seed=2)
    _, m0, _ = s.dispatch(G, T, [5, 6])
    assert s.dispatch(G, T, [x for x in (5, 6) if x != m0])[1] == m0


def test_round_robin_walks_the_members_and_skips_failures():
    s = SharedSub("round_robin", seed=4)
    members = [1, 2, 3, 4]
    seq = [s.dispatch(G, T, members)[1] for _ in range(8)]
    start = members.index(seq[0])
    assert seq == [members[(start + k) % 4] for k in range(8)]
    # a failure: the next member of the remaining ones (the counter indexes the list it picks from)
    res, m, failed = s.dispatch(G, T, members, qos=1, ack_enabled=True, respond=lambda x: "nack" if x == 1 else "ack")
    assert res == ("ok", 1) and m != 1 and failed in ([], [1])


@pytest.mark.parametrize("strategy", ["hash", "hash_clientid", "hash_topic"])
def test_hash_strategies_are_stable_per_key(strategy):
    s = SharedSub(strategy)
    members = list(range(20))
    a = [s.dispatch(G, T, members, b"s/%d" % k, b"c%d" % k)[1] for k in range(30)]
    b = [s.dispatch(G, T, members, b"s/%d" % k, b"c%d" % k)[1] for k in range(30)]
    assert a == b


def test_unknown_strategy_is_refused():
    with pytest.raises(ValueError):
        SharedSub("lowest_latency")
