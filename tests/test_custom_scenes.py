"""Kernel choice and stream layout on scenes built through the ABI's constructors (tests/scenes.py).

ADVICE r03:
- a sphere-only scene with Lists inside BvhNodes gets the GENERAL walk stream (a List's members are tested
  under their enclosing BvhNode box once, list.rs:20-31 / bvh_node.rs:104-127); plan() must then send it to
  the general kernels, not the sphere kernel (render.hip plan);
- a group's box-less leaves must be contiguous in the leaf sequence (lane.h gstate keeps one group), so a
  List around a nested BvhNode of its own Lists keeps the outer box whole (scene.cpp gwalk_leaves_grouped);
- a textured sphere scene whose walk stream exceeds the LDS budget runs the HEAVY walk over the staged
  part plus global memory (render_sphere.hip launch_sphere), not over LDS it does not own.
CPU tests check the stream; -m gpu tests hold the default path to the verbatim reference traversal bit for bit.
"""
import numpy as np
import pytest

import hrt
import scenes


def _groups_contiguous(leaves):
    seen, cur = set(), None
    for _, _, flags, g in leaves:
        if not flags & scenes.GL_BOX or g == cur:
            continue
        if g in seen:
            return False
        if cur is not None:
            seen.add(cur)
        cur = g
    return True


def test_sphere_lists_get_the_general_stream():
    s = scenes.sphere_lists()
    blob, info = hrt.scene_blob(s)
    assert info.walk_bytes > 0 and info.walk_general == 1
    leaves = scenes.general_stream_leaves(blob, info)
    assert any(f & scenes.GL_BOX for _, _, f, _ in leaves)  # box-less List members under a group box
    assert _groups_contiguous(leaves)


def _nested():
    s = hrt.Scene()
    m = s.lambertian(s.solid(0.5, 0.5, 0.5))
    sp = [s.sphere((x * 0.5, 0.2, 0.0), 0.2, m) for x in range(7)]
    inner = s.bvh([s.list([sp[1], s.bvh([sp[2], sp[3]])]), sp[4]])
    outer = s.bvh([s.list([sp[0], inner, sp[5]]), sp[6]])
    s.set_root(s.bvh([outer, s.sphere((0, -1000, 0), 1000, m)]))
    return s


def test_nested_list_group_kept_whole(monkeypatch):
    """A BvhNode leaf holding List [a, BvhNode(Leaf(List[c, BvhNode[d, e]]), g), f]: a and f are box-less
    members of the outer group, c of the inner one.  Without the fallback (HRT_GWALK_GROUPED=0) the outer
    group's leaves straddle the inner group's; with it, every group's leaves are contiguous."""
    monkeypatch.setenv("HRT_GWALK_GROUPED", "0")
    blob, info = hrt.scene_blob(_nested())
    assert info.walk_general == 1 and not _groups_contiguous(scenes.general_stream_leaves(blob, info))
    monkeypatch.delenv("HRT_GWALK_GROUPED")
    blob, info = hrt.scene_blob(_nested())
    assert _groups_contiguous(scenes.general_stream_leaves(blob, info))


def test_big_textured_stream_is_beyond_lds():
    s = scenes.big_textured()
    _, info = hrt.scene_blob(s)
    assert info.walk_general == 0 and info.walk_hot > 0 and info.walk_bytes > info.walk_hot


def _reference_equal(s, w, h, spp, monkeypatch, kernels=("segment",)):
    s.commit()
    cam = scenes.camera(w, h)
    p = hrt.params(w, h, spp, 50, 11)
    a, sa = hrt.render(s, cam, p, stats=True)
    ref, sr = hrt.render(s, cam, hrt.params(w, h, spp, 50, 11, flags=hrt.RENDER_REFERENCE_CULL), stats=True)
    assert sa.segments == sr.segments
    assert np.array_equal(a, ref)
    for k in kernels:
        monkeypatch.setenv("HRT_KERNEL", k)
        b, sb = hrt.render(s, cam, p, stats=True)
        monkeypatch.delenv("HRT_KERNEL")
        assert sb.segments == sa.segments and np.array_equal(a, b), k
    assert np.isfinite(a).all()
    return a, sa


@pytest.mark.gpu
def test_sphere_lists_on_gpu_equal_reference_traversal(monkeypatch):
    a, st = _reference_equal(scenes.sphere_lists(), 160, 90, 24, monkeypatch, ("segment", "persistent"))
    assert st.prim_slots == 0  # counters off; the default ran the general walk kernel (no sphere payload reads)


@pytest.mark.gpu
def test_big_textured_hybrid_heavy_equals_reference_traversal(monkeypatch):
    s = scenes.big_textured()
    _reference_equal(s, 160, 90, 16, monkeypatch)
    assert s.scene_info().in_lds == 2  # the stream's staged part in LDS, the rest in global memory


@pytest.mark.gpu
def test_foggy_media_shapes_equal_reference_traversal(monkeypatch):
    """Every medium shape of the general walk stream (flat one-sphere and moving-sphere media, a box-less List
    member, a Cuboid boundary, a fog around the scene) on the GPU: the general walk kernel bit for bit equal to
    the verbatim reference traversal and to the segment kernel (tests/test_lane_sim.py runs the same on the
    host lanes)."""
    _reference_equal(scenes.foggy(), 120, 72, 16, monkeypatch, ("segment",))
