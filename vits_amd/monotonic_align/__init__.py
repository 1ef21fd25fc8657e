"""Drop-in for the external ``monotonic_align`` package the reference imports
(models.py:12-15, called at models.py:498).

``maximum_path(neg_cent, mask)`` keeps the published contract — neg_cent
[b, t_t, t_s] scores, mask [b, t_t, t_s], returns a 0/1 path tensor of
neg_cent's dtype on neg_cent's device — but runs the DP and backtrack on the
GPU (vits_maximum_path in libvits_amd), asynchronously on the current stream,
with no device->host->device round trip.  Bit-exact against the Cython core
(the DP is fp32 add/max only); see vits_amd/csrc/mas.hip.
"""
from ..ops import maximum_path, maximum_path_lengths

__all__ = ["maximum_path", "maximum_path_lengths"]
