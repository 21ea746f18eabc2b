"""Arena / gating: drop-in for the commented arena of exp/learner.py:97-145.

The reference's learner once played the new network against the previous one: its agent
first (RoundRobinReferee((new, old)): new moves first) then second, counted decisive games with
WinnerRecorder (exp/callbacks.py:7-28), and returned new_wins / (new_wins + old_wins + 1e-8);
LearnPuppet.update kept the new weights when that exceeded 0.55 (app/base.py:194-196, also
commented).  Here both sides run as batched engine play: the engine holds the two networks in
its two weight slots and each move's leaves are evaluated with the network of the agent to move
(mtaz_set_agent_slots).  All games of a side run in lockstep, so one launch per simulation wave
still covers every game.
"""
import numpy as np

ARENA_GAME_NUMBER_PER_SIDE = 3      # exp/learner.py:18
GATE = 0.55                         # app/base.py:195
DECISIVE = 1                        # csrc/rules.h Outcome


def winners(records):
    """WinnerRecorder.results over the games of one play(): {False: agent 0 wins, True: agent 1
    wins}; a decisive game is won by the agent that made the last move (exp/callbacks.py:19-22:
    winner = not referee.turn), draws are not counted."""
    res = {False: 0, True: 0}
    for plies, outcome in zip(records['plies'], records['outcome']):
        if int(outcome) == DECISIVE:
            res[bool((int(plies) - 1) % 2)] += 1
    return res


def arena(engine, new_net, old_net, seed_base=0):
    """Play engine.G games with the new network moving first and engine.G with it moving second.
    Returns {'new_wins', 'old_wins', 'draws', 'score'} with score as exp/learner.py:145.
    Afterwards weight slot 0 holds new_net and self-play (both agents on slot 0) is restored."""
    engine.set_weights(new_net, slot=0)
    engine.set_weights(old_net, slot=1)
    out = {'new_wins': 0, 'old_wins': 0, 'draws': 0, 'games': 0}
    try:
        for side, (s0, s1) in enumerate(((0, 1), (1, 0))):        # new first, then new second
            engine.set_agent_networks(s0, s1)
            engine.set_seed_base(seed_base + side * engine.G)
            engine.play()
            rec = engine.records()
            w = winners(rec)
            new_first = side == 0
            out['new_wins'] += w[False] if new_first else w[True]
            out['old_wins'] += w[True] if new_first else w[False]
            out['draws'] += int(np.sum(rec['outcome'] != DECISIVE))
            out['games'] += len(rec['plies'])
    finally:
        engine.set_agent_networks(0, 0)
    out['score'] = out['new_wins'] / (out['new_wins'] + out['old_wins'] + 1e-8)
    return out


def gate(score, threshold=GATE):
    """Keep the new network when it scored above the threshold (app/base.py:195-196)."""
    return score > threshold
