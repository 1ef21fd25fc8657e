"""GAN / KL losses (reference ``losses.py``): small reductions, host-side torch.

``discriminator_loss`` returns per-discriminator losses as device tensors
instead of calling ``.item()`` inside the loop (losses.py:28-29), so the
training step does not sync the host once per discriminator; call
``float()`` on them when logging.
"""
import torch


def feature_loss(fmap_r, fmap_g):
    loss = 0
    for dr, dg in zip(fmap_r, fmap_g):
        for rl, gl in zip(dr, dg):
            loss = loss + torch.mean(torch.abs(rl.float().detach() - gl.float()))
    return loss * 2


_SEG = {}


def _segments(outs):
    """(flat fp32 weights 1/N_i per element, int64 segment ids) of a list of
    tensors, cached per (shapes, device)."""
    key = (tuple(tuple(o.shape) for o in outs), str(outs[0].device))
    if key not in _SEG:
        sizes = [o.numel() for o in outs]
        w = torch.cat([torch.full((n,), 1.0 / n) for n in sizes]).to(outs[0].device)
        seg = torch.cat([torch.full((n,), i, dtype=torch.long)
                         for i, n in enumerate(sizes)]).to(outs[0].device)
        _SEG[key] = (w, seg)
    return _SEG[key]


def _flat(outs):
    """All the discriminator outputs as one fp32 vector (one cat in their own
    dtype, one cast) instead of a cast and three reductions per output."""
    return torch.cat([o.reshape(-1) for o in outs]).float()


def _per_output(terms, seg, n):
    return list(torch.zeros(n, device=terms.device, dtype=terms.dtype)
                .index_add_(0, seg, terms.detach()).unbind(0))


def discriminator_loss(disc_real_outputs, disc_generated_outputs):
    """sum_i mean((1 - dr_i)^2) + mean(dg_i^2) (losses.py:17-30), each
    output's mean as a weighted sum (weights 1/N_i) over the concatenated
    outputs: a few launches for all ten discriminator heads instead of ~8
    per head each way."""
    n = len(disc_real_outputs)
    wr, sr = _segments(disc_real_outputs)
    wg, sg = _segments(disc_generated_outputs)
    r = (1 - _flat(disc_real_outputs)) ** 2 * wr
    g = _flat(disc_generated_outputs) ** 2 * wg
    loss = r.sum() + g.sum()
    return loss, _per_output(r, sr, n), _per_output(g, sg, n)


def generator_loss(disc_outputs):
    """sum_i mean((1 - dg_i)^2) (losses.py:33-42) over the concatenated
    outputs (see discriminator_loss); the per-head losses are returned
    detached (the reference returns them for logging only)."""
    w, s = _segments(disc_outputs)
    t = (1 - _flat(disc_outputs)) ** 2 * w
    return t.sum(), _per_output(t, s, len(disc_outputs))


def kl_loss(z_p, logs_q, m_p, logs_p, z_mask):
    """KL term of losses.py:46-61 (fp32)."""
    z_p, logs_q, m_p, logs_p, z_mask = (t.float() for t in (z_p, logs_q, m_p, logs_p, z_mask))
    kl = logs_p - logs_q - 0.5
    kl = kl + 0.5 * ((z_p - m_p) ** 2) * torch.exp(-2.0 * logs_p)
    return torch.sum(kl * z_mask) / torch.sum(z_mask)
