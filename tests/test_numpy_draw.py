"""Host side of EmoVITS graph mode's noise-slice draw (CPU).

infer.py:173 draws ``np.random.randint(noise.size(0) - nl)`` after y_len is
known.  In graph mode y_len only exists on the device, so the host hands the
kernel (misc.hip expand_durations_kernel, noise_mode 1) a pool of raw
MT19937 words from numpy's global generator (ops.numpy_draw_pool); the
kernel picks the start with numpy's legacy masked rejection and reports how
many words it consumed, and ops.numpy_draw_commit re-advances the generator
by that many.  ``_device_select`` restates the kernel's selection line by
line; together they must reproduce randint's value AND its generator state
for every range, which is what this test pins against numpy itself."""
import numpy as np

from vits_amd import ops


def _device_select(words: np.ndarray, high: int):
    """misc.hip expand_durations_kernel, mode 1 (returns start, used)."""
    if high < 1 or high - 1 > 0xFFFFFFFF:
        return 0, -1
    rng = high - 1
    if rng == 0:
        return 0, 0
    mask = rng
    for sh in (1, 2, 4, 8, 16):
        mask |= mask >> sh
    for i, w in enumerate(words.view(np.uint32)):
        if (int(w) & mask) <= rng:
            return int(w) & mask, i + 1
    return 0, -2  # every word of the pool rejected: the host advances and retries


def test_device_draw_reproduces_numpy_randint_and_state():
    highs = [1, 2, 3, 5, 7, 8, 9, 255, 256, 257, 1000, 65535, 65536, 65537,
             192 * 4096 - 192 * 37, 786432 - 1, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 1, 2 ** 32]
    highs += list(np.random.default_rng(5).integers(1, 2 ** 31, 40))
    for seed, high in enumerate(highs):
        high = int(high)
        np.random.seed(seed)
        want = np.random.randint(high)
        want_next = np.random.randint(1 << 30)
        np.random.seed(seed)
        pool, state = ops.numpy_draw_pool()
        start, used = _device_select(pool, high)
        assert used >= 0, high
        ops.numpy_draw_commit(state, used)
        assert start == want, (high, start, want)
        assert np.random.randint(1 << 30) == want_next, high


def test_device_draw_rejects_slices_that_do_not_fit():
    pool, state = ops.numpy_draw_pool()
    assert _device_select(pool, 0)[1] == -1
    assert _device_select(pool, -5)[1] == -1


def _host_draw(high: int, n: int):
    """infer.py EmoVITS._infer_graph's draw protocol (vits_amd/infer.py:200-214)
    with a pool of ``n`` words: -2 (all rejected) advances numpy's generator
    past the pool and draws again from the next words."""
    while True:
        pool, state = ops.numpy_draw_pool(n)
        start, used = _device_select(pool, high)
        if used == -2:
            ops.numpy_draw_commit(state, n)
            continue
        assert used >= 0
        ops.numpy_draw_commit(state, used)
        return start


def test_device_draw_all_rejected_pool_retries_in_step_with_numpy():
    """Pools of 1-3 words at ranges whose masked rejection rate is ~1/2, so
    whole pools are rejected often: the retry must still give randint's value
    and leave the generator where randint leaves it."""
    retries = 0
    for seed in range(60):
        for high in (2 ** 31 + 1, 2 ** 16 + 1, 5):
            for n in (1, 2, 3):
                np.random.seed(seed)
                want = np.random.randint(high)
                want_next = np.random.randint(1 << 30)
                np.random.seed(seed)
                pool, _ = ops.numpy_draw_pool(n)
                retries += _device_select(pool, high)[1] == -2
                np.random.seed(seed)
                assert _host_draw(high, n) == want, (seed, high, n)
                assert np.random.randint(1 << 30) == want_next, (seed, high, n)
    assert retries > 20  # the -2 branch was exercised
