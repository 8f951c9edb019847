"""What may change an image's bits is explicit configuration (hrt_scene_options), never the environment
(the reference takes its configuration as arguments, src/arguments.rs:23-47):
  - the library reads the environment only through knob_env (csrc/knobs.cpp), and only A/B knobs between
    bit-identical variants, each listed in KNOWN_KNOBS (hrt_last_launch reports the set ones);
  - the retired output-changing variables (HRT_CHUNK_MIN/DIV/TAIL, HRT_WALK_TREE, HRT_BVH_TIES) no longer
    change the chunk schedule or the flattened scene; the options do;
  - the partial-sum budget caps the chunk count by the full image size, leaving every
    BASELINE configuration's schedule as it was.
CPU only: the chunk schedule and the flattened scene are host computations (hrt_debug_sample_chunks,
hrt_debug_scene_blob); tests/test_gpu_parity.py::test_env_chunk_knobs_do_not_change_frame renders."""
import os
import re

import pytest

import hrt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hyper-ray-tracer_amd", "csrc")
RETIRED = {"HRT_CHUNK_MIN": "1", "HRT_CHUNK_DIV": "512", "HRT_CHUNK_TAIL": "0", "HRT_WALK_TREE": "reference",
           "HRT_BVH_TIES": "reverse"}


def _sources():
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".cpp", ".hip", ".h", ".hpp")):
            yield f, open(os.path.join(CSRC, f)).read()


def test_environment_is_read_only_through_knob_env():
    table = re.search(r"KNOWN_KNOBS\[\]\s*=\s*\{(.*?)\};", open(os.path.join(CSRC, "knobs.cpp")).read(), flags=re.S).group(1)
    known = re.findall(r'"(HRT_\w+)"', table)
    assert len(known) > 10
    read = set()
    for f, src in _sources():
        code = re.sub(r"/\*.*?\*/|//[^\n]*", "", src, flags=re.S)
        if f != "knobs.cpp":
            assert "getenv" not in code, f"{f} reads the environment outside knobs.cpp"
        read |= set(re.findall(r'knob_env\("(HRT_\w+)"\)', code))
    read |= {n for n in re.findall(r'env_knob\("(HRT_\w+)"', "".join(s for _, s in _sources()))}
    assert read <= set(known), read - set(known)
    assert not set(known) & set(RETIRED), "an output-changing variable is still an environment knob"


def _chunks(name, W, H, spp, monkeypatch=None, env=None, **opts):
    if env:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
    s = hrt.preset(name, 1, None, options=opts or None)
    c = hrt.sample_chunks(s, hrt.params(W, H, spp, 50, 1, tuple(s.info.background)))
    if env:
        for k in env:
            monkeypatch.delenv(k)
    return c


@pytest.mark.parametrize("name,W,H,spp", [("random", 1920, 1080, 500), ("cornell", 2048, 2048, 10000),
                                          ("final", 800, 800, 64)])
def test_retired_chunk_variables_no_longer_change_the_schedule(name, W, H, spp, monkeypatch):
    base = _chunks(name, W, H, spp)
    assert _chunks(name, W, H, spp, monkeypatch, RETIRED) == base
    # the explicit options do change it
    assert _chunks(name, W, H, spp, chunk_min=2 * base["chunk"]) != base
    if base["tail"]:
        assert _chunks(name, W, H, spp, chunk_uniform=1)["tail"] == 0
    assert _chunks(name, W, H, spp, chunk_min=spp) == {"chunk": spp, "head": 1, "first": spp, "tail": 0}


def test_chunk_schedules_of_the_baseline_configs():
    """The sample chunks each BASELINE configuration sums in (the budget below leaves them alone)."""
    got = {k: _chunks(*k) for k in [("random", 1920, 1080, 500), ("earth_perlin", 1920, 1080, 1000),
                                     ("random_10k", 3840, 2160, 2000), ("cornell", 2048, 2048, 10000)]}
    assert got[("random", 1920, 1080, 500)]["chunk"] == 16
    assert got[("random_10k", 3840, 2160, 2000)] == {"chunk": 63, "head": 30, "first": 59, "tail": 10}
    for (name, W, H, spp), c in got.items():
        n = c["head"] + c["tail"]
        assert n * W * H * 16 <= 6 << 30
        # the samples add up: first + (head - 1) * chunk + the halving tail
        tail = sum(c["chunk"] >> (1 + (j >> 1)) for j in range(c["tail"]))
        assert c["first"] + (c["head"] - 1) * c["chunk"] + tail == spp, (name, c)


def test_partial_budget_caps_chunks_by_frame_size():
    """deep general scenes take one-sample chunks (up to 64 per pixel); at 3840x2160 that is
    8.5 GB of partial sums per launch in flight.  The cap doubles the chunk until n_chunks x W x H x 16 B fits
    6 GiB; it depends on the full image only, so every tile split of a frame keeps one schedule."""
    small = _chunks("final", 800, 800, 64)
    assert small == {"chunk": 1, "head": 64, "first": 1, "tail": 0}
    big = _chunks("final", 3840, 2160, 64)
    n = big["head"] + big["tail"]
    assert n * 3840 * 2160 * 16 <= 6 << 30 and big == {"chunk": 2, "head": 31, "first": 2, "tail": 2}


def test_retired_scene_variables_no_longer_change_the_flattened_scene(monkeypatch):
    """HRT_BVH_TIES / HRT_WALK_TREE in the environment: the same blob byte for byte; the options change it
    (final: 31 sorts with tied keys; random: its walk hierarchy)."""
    earth = hrt.synthetic_earth()
    for name in ("final", "random"):
        base = bytes(hrt.scene_blob(hrt.preset(name, 1, earth))[0])
        for k, v in RETIRED.items():
            monkeypatch.setenv(k, v)
        again = bytes(hrt.scene_blob(hrt.preset(name, 1, earth))[0])
        for k in RETIRED:
            monkeypatch.delenv(k)
        assert again == base, name
    ties = hrt.scene_blob(hrt.preset("final", 1, earth, options={"bvh_ties": 1}))
    assert bytes(ties[0]) != bytes(hrt.scene_blob(hrt.preset("final", 1, earth))[0]) and ties[1].bvh_tied_sorts > 0
    tree = hrt.scene_blob(hrt.preset("random", 1, earth, options={"walk_tree": 1}))
    assert tree[1].walk_regrouped == 0


def test_options_round_trip_and_reject_bad_values():
    s = hrt.Scene()
    assert tuple(getattr(s.options(), f) for f, _ in hrt.SceneOptions._fields_) == (0, 0, 0, 0, 0)
    s.set_options(chunk_min=8, walk_tree=1)
    o = s.options()
    assert (o.chunk_min, o.walk_tree, o.bvh_ties) == (8, 1, 0)
    with pytest.raises(hrt.HrtError) as e:
        s.set_options(bvh_ties=2)
    assert e.value.status == hrt.ERR_INVALID_ARG
    with pytest.raises(TypeError):
        s.set_options(chunk_tail=3)


def test_view_hint_places_only_and_clears():
    """hrt_scene_set_view is a placement hint: it changes which node parts of random_10k's stream (beyond LDS)
    are staged, NULL restores the default placement byte for byte, and it is refused after commit like every
    other scene setting (the commit needs a device, so the refusal is checked on the uncommitted path)."""
    def walk(s):
        b, i = hrt.scene_blob(s)
        return bytes(b)[i.off_walk:i.off_walk + i.walk_bytes], i.walk_hot

    s0 = hrt.preset("random_10k", 1, None)
    base, hot0 = walk(s0)
    s1 = hrt.preset("random_10k", 1, None)
    s1.set_view(hrt.preset_camera(s1.info, 3840, 2160))
    viewed, hot1 = walk(s1)
    assert hot0 == hot1 > 0 and viewed != base and len(viewed) == len(base)
    s2 = hrt.preset("random_10k", 1, None)
    s2.set_view(hrt.preset_camera(s2.info, 3840, 2160))
    s2.set_view(None)
    assert walk(s2)[0] == base
    # a stream staged whole (Random) has no placement choice; its re-grouped hierarchy does weigh the view's rays
    # (walk_regroup_dp), and with the reference tree itself (walk_tree 1) the view changes nothing
    s3 = hrt.preset("random", 1, None)
    b3, h3 = walk(s3)
    s3b = hrt.preset("random", 1, None)
    s3b.set_view(hrt.preset_camera(s3b.info, 1920, 1080))
    b3b, h3b = walk(s3b)
    assert h3 == h3b == 0 and len(b3b) == len(b3) and b3b != b3
    t0 = hrt.preset("random", 1, None, options={"walk_tree": 1})
    t1 = hrt.preset("random", 1, None, options={"walk_tree": 1})
    t1.set_view(hrt.preset_camera(t1.info, 1920, 1080))
    assert walk(t0)[0] == walk(t1)[0]
