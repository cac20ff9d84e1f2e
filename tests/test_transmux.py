"""Batched transmux stage (decrypt + demux between FRAG_LOADED and the buffer): every
fragment's result — status, info row, plaintext length, video/audio/id3 ES views — matches
the per-segment host oracle, for a mixed batch (encrypted + clear, varied sizes, one bad
key) staged from host payloads.  Runs on CPU (host kernels) and on the GPU (HIP kernels)."""
import pytest
import torch

from hlsjs_p2p_wrapper_amd.net import new_event_loop
from hlsjs_p2p_wrapper_amd.ops import aes, tsdemux
from hlsjs_p2p_wrapper_amd.player.transmux import InfoRow, MediaPipeline, TransmuxJob


def _batch():
    key = bytes(range(16))
    jobs = []
    for i, (nbytes, enc) in enumerate([(300_000, True), (188 * 700, False), (1_000_000, True), (50_000, True),
                                       (188 * 64, False)]):
        seg, st = tsdemux.mux_segment(duration=2.0, target_bytes=nbytes, with_id3=(i % 2 == 0), seed=10 + i, sn=i)
        iv = aes.iv_from_sn(i)
        payload = aes.cbc_encrypt(key, iv, seg) if enc else seg
        jobs.append((seg, payload, key if enc else None, iv if enc else None))
    return jobs


def _run(device):
    loop = new_event_loop("virtual")
    pipe = MediaPipeline(torch.device(device), loop)
    out = {}
    jobs = _batch()
    for n, (_, payload, key, iv) in enumerate(jobs):
        pipe.submit(TransmuxJob(torch.from_numpy(payload.copy()), key, iv, lambda r, n=n: out.__setitem__(n, r)))
    bad = jobs[0]
    pipe.submit(TransmuxJob(torch.from_numpy(bad[1].copy()), bytes(16), bad[3], lambda r: out.__setitem__("bad", r)))
    pipe.flush()
    return jobs, out


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_pipeline_results_match_oracle(device, request):
    if device == "cuda":
        request.getfixturevalue("cuda")
    jobs, out = _run(device)
    for n, (seg, _, _, _) in enumerate(jobs):
        r = out[n]
        assert r.get("error") is None and r["status"] == 0
        assert r["plain_bytes"] == len(seg)
        ref = tsdemux.demux_batch(torch.from_numpy(seg.copy()), [0], [len(seg)],
                                  torch.zeros(len(seg) + 256, dtype=torch.uint8), [0]).segment(0)
        info = r["info"]
        assert isinstance(info, InfoRow)
        for k in ("video_pid", "audio_pid", "video_bytes", "audio_bytes", "id3_bytes", "n_video_pes",
                  "video_first_pts", "video_last_pts"):
            assert info[k] == ref[k], k
        assert torch.equal(r["video"].cpu(), ref["video"]["es"])
        assert torch.equal(r["audio"].cpu(), ref["audio"]["es"])
        assert r["id3"].numel() == ref["id3_bytes"]
        assert info.to_dict()["video_bytes"] == ref["video_bytes"] and "status" in info
    # wrong key: bad padding (overwhelmingly likely) or garbage that fails demux
    bad = out["bad"]
    assert bad.get("error") is not None or bad["status"] != 0
