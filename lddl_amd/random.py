"""RNG-state passing wrappers (lddl/random.py:28-55): each call runs CPython's `random` on an
explicit state and returns the advanced state, leaving the global generator untouched."""
import random


def _run(fn, rng_state):
    r = random.Random()
    r.setstate(rng_state)
    out = fn(r)
    return out, r.getstate()


def randrange(stop, rng_state=None):
    return _run(lambda r: r.randrange(stop), rng_state)


def shuffle(x, rng_state=None):
    return _run(lambda r: r.shuffle(x), rng_state)[1]


def sample(population, k, rng_state=None):
    return _run(lambda r: r.sample(population, k), rng_state)


def choices(population, weights=None, cum_weights=None, k=1, rng_state=None):
    return _run(lambda r: r.choices(population, weights=weights, cum_weights=cum_weights, k=k),
                rng_state)


def seeded_state(seed):
    """random.seed(seed); random.getstate() without touching the global generator."""
    return random.Random(seed).getstate()
