"""The multi-GPU gather through the C-ABI (eray_gather_rows over an RCCL communicator from
eray_comm_init), on the one GPU of the box: a one-rank communicator gathers a rendered block into
the frame buffer (and in place).  More ranks need one GPU each (RCCL puts one rank per device):
the 2-rank split and gather order are covered on CPU (tests/test_dist_rows.py) and the tiles'
pixels on the GPU (tests/test_gpu_configs.py).  The banded gather's coded transport (uniform
64-pixel segments as one word, comm.cpp) is checked here rank by rank: N ranks' padded blocks
encoded into rank 0's layout and decoded (eray_debug_coded_unband) against the plain reorder and a
numpy restatement of the band split."""
import numpy as np
import pytest

from eray_amd import capi
from eray_amd.frame import MainScene

pytestmark = pytest.mark.gpu


def test_one_rank_gather_through_rccl(gpu, cube):
    W, H = 256, 144
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    local = gpu.empty((H, W, 3), np.uint8)
    frame = gpu.empty((H, W, 3), np.uint8)
    comm = None
    try:
        gpu.memset(frame.ptr, 0, frame.nbytes)
        gpu.render(W, H, out_ppm=local.ptr)
        comm = gpu.comm_init(1, 0, capi.comm_unique_id())
        gpu.gather_rows(comm, local.ptr, frame.ptr, H, W)
        gpu.synchronize()
        want = local.numpy()
        assert (want != 0).any()
        assert np.array_equal(frame.numpy(), want)
        gpu.gather_rows(comm, local.ptr, local.ptr, H, W)  # in place
        gpu.synchronize()
        assert np.array_equal(local.numpy(), want)
        with pytest.raises(capi.ErayError):
            gpu.gather_rows(comm, local.ptr, None, H, W)  # rank 0 needs the frame
    finally:
        if comm:
            capi.comm_destroy(comm)
        local.free()
        frame.free()
        sc.close()


def _banded_blocks(frame, H, W, band, world):
    """Each rank's padded local PPM block (local file order) of a file-order frame, as
    eray_render writes it for dist.band_split (numpy restatement of eray_band_rows' split)."""
    cam = frame[::-1]  # camera rows
    rows_max = capi.band_rows(H, band, world, 0)  # rank 0 holds the most rows (the padded size)
    blocks = np.zeros((world, rows_max, W, 3), np.uint8)
    for r in range(world):
        mine = [y for y in range(H) if (y // band) % world == r]
        assert len(mine) == capi.band_rows(H, band, world, r)
        blocks[r, :len(mine)] = cam[mine][::-1]
    return blocks


@pytest.mark.parametrize("W,H,band,world", [(192, 64, 4, 1), (192, 64, 4, 2), (208, 68, 4, 3), (37, 40, 8, 2),
                                            (1920, 120, 4, 8), (70, 12, 4, 5), (64, 30, 4, 3),
                                            (64, 26, 4, 3)])  # the short tail band on rank 0
def test_coded_banded_gather_layout(gpu, W, H, band, world):
    rng = np.random.default_rng(W * 7 + H + world)
    frame = np.empty((H, W, 3), np.uint8)
    frame[:] = (25, 25, 51)  # mostly the miss colour, uniform segments
    for _ in range(6):  # patches of noise (non-uniform segments), some at the right edge
        y, x = rng.integers(0, H), rng.integers(0, W)
        frame[y:y + rng.integers(1, 9), x:x + rng.integers(1, 90)] = rng.integers(0, 256, (1, 1, 3), dtype=np.uint8)
        frame[y, x] = rng.integers(0, 256, 3, dtype=np.uint8)
    frame[H // 2, :] = rng.integers(0, 256, (W, 3), dtype=np.uint8)
    frame[1] = (7, 8, 9)  # a uniform row of another colour
    blocks = _banded_blocks(frame, H, W, band, world)
    assert blocks.shape[1] == capi.lib().eray_band_rows(H, band, world, 0)
    staging = gpu.to_device(np.ascontiguousarray(blocks))
    out = gpu.empty((H, W, 3), np.uint8)
    try:
        for fn in ("eray_debug_unband", "eray_debug_coded_unband"):
            gpu.memset(out.ptr, 0, out.nbytes)
            assert getattr(capi.lib(), fn)(gpu.handle, staging.ptr, out.ptr, H, W, band, world) == 0
            gpu.synchronize()
            assert np.array_equal(out.numpy(), frame), fn
    finally:
        staging.free()
        out.free()


def test_one_rank_banded_gather_through_rccl(gpu, cube):
    """eray_gather_rows with bands on a one-rank communicator: the coded transport end to end
    (encode, the count all-gather, decode) gives the rendered frame."""
    W, H = 320, 180
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    local = gpu.empty((H, W, 3), np.uint8)
    frame = gpu.empty((H, W, 3), np.uint8)
    comm = None
    try:
        gpu.render(W, H, out_ppm=local.ptr)
        comm = gpu.comm_init(1, 0, capi.comm_unique_id())
        for band in (4, 8):
            gpu.memset(frame.ptr, 0, frame.nbytes)
            gpu.gather_rows(comm, local.ptr, frame.ptr, H, W, band_rows=band)
            gpu.synchronize()
            assert np.array_equal(frame.numpy(), local.numpy()), band
    finally:
        if comm:
            capi.comm_destroy(comm)
        local.free()
        frame.free()
        sc.close()


def _blocks_of(frame, H, W, band, world):
    """Each rank's padded local PPM rows of a file-order frame: interleaved bands, or (band 0)
    the rank's block of file rows."""
    if band:
        return _banded_blocks(frame, H, W, band, world)
    h = H // world
    return np.ascontiguousarray(frame.reshape(world, h, W, 3))


@pytest.fixture(scope="module")
def standin70k_gather():
    from eray_amd import meshgen
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


@pytest.mark.parametrize("mesh", ["cube", "standin70k"])
def test_scene_camera_gather_layout(gpu, cube, standin70k_gather, mesh):
    """The scene-camera gather (only the objects' pixel rectangles travel, comm.cpp) of N ranks
    simulated on one GPU: every rank's rows packed with its own rectangles, then assembled — the
    frame must be the rendered frame, byte for byte, for bands and blocks."""
    W, H = (320, 180) if mesh == "cube" else (480, 270)
    sc = MainScene(gpu, *(cube if mesh == "cube" else standin70k_gather), W, H, texture=64, fov=(16.0, 9.0))
    ppm = gpu.empty((H, W, 3), np.uint8)
    out = gpu.empty((H, W, 3), np.uint8)
    try:
        gpu.render(W, H, out_ppm=ppm.ptr)
        frame = ppm.numpy()
        assert (frame != np.array([25, 25, 51], np.uint8)).any()
        for world in (1, 2, 3, 5, 8):
            for band in (0, 4, 8):
                if not band and H % world:
                    continue
                blocks = _blocks_of(frame, H, W, band, world)
                staging = gpu.to_device(blocks)
                try:
                    gpu.memset(out.ptr, 0, out.nbytes)
                    assert capi.lib().eray_debug_scene_gather(gpu.handle, staging.ptr, out.ptr, H, W, band, world) == 0
                    assert np.array_equal(out.numpy(), frame), (world, band)
                finally:
                    staging.free()
    finally:
        ppm.free()
        out.free()
        sc.close()


def test_scene_camera_gather_batch_rotating_roots(gpu, cube):
    """A batch of B different frames through N simulated ranks (real pack and assembly kernels,
    each rank's transfer schedule played as device copies): with rank 0 assembling every frame and
    with ERAY_GATHER_ROTATE_ROOT (frame k on rank k % N, root r's frames contiguous in root
    order), every assembled frame is the frame the ranks rendered — the same bytes either way."""
    W, H = 320, 180
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    ppm = gpu.empty((H, W, 3), np.uint8)
    try:
        gpu.render(W, H, out_ppm=ppm.ptr)
        base = ppm.numpy()
        for world, B, band in ((1, 3, 4), (2, 5, 4), (3, 7, 8), (4, 4, 4), (8, 11, 4), (8, 3, 4), (5, 9, 0)):
            if not band and H % world:
                continue
            # frame k: the rendered frame with every byte shifted by 37 k (inside the rectangles
            # only those bytes travel; outside, the assembly writes the miss colour)
            fr = [(base.astype(np.int32) + 37 * k).astype(np.uint8) for k in range(B)]
            blocks = np.stack([_blocks_of(f, H, W, band, world) for f in fr])  # [k][q] rows
            staging = gpu.to_device(np.ascontiguousarray(blocks))
            out = gpu.empty((B, H, W, 3), np.uint8)
            try:
                got = {}
                for rotate in (0, 1):
                    gpu.memset(out.ptr, 0, out.nbytes)
                    assert capi.lib().eray_debug_scene_gather_batch(gpu.handle, staging.ptr, out.ptr, B, H, W, band,
                                                                    world, rotate) == 0
                    got[rotate] = out.numpy()
                assert np.array_equal(got[0][0], base), (world, B, band)
                order = [k for r in range(world) for k in range(r, B, world)]  # root-grouped batch order
                for pos, k in enumerate(order):
                    assert np.array_equal(got[1][pos], got[0][k]), (world, B, band, k)
                assert not np.array_equal(got[0][0], got[0][B - 1])
            finally:
                staging.free()
                out.free()
    finally:
        ppm.free()
        sc.close()


def test_one_rank_gather_frames_and_graph_capture(cube):
    """eray_gather_frames on a one-rank communicator: a ring of rendered frames, gathered per
    frame (coded path) and scene-camera style, then the scene-camera gather captured in a HIP
    graph (torch.cuda.CUDAGraph on the context's stream) and replayed — no host synchronisation
    inside, so the capture succeeds and the replay assembles the frames again."""
    import torch
    W, H, S = 320, 180, 4
    st = torch.cuda.Stream()
    gpu = capi.Context(0)  # its own context: the stream below outlives nothing else
    gpu.set_stream(st.cuda_stream)
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    ring = capi.frame_ring(S, H, W)
    rgb = gpu.empty((S, H, W, 3), np.float32)
    local = gpu.empty((S, H, W, 3), np.uint8)
    frames = gpu.empty((S, H, W, 3), np.uint8)
    comm = None
    try:
        gpu.render_frames(S, W, H, out_rgb=rgb.ptr, out_ppm=local.ptr, ring=ring)
        gpu.synchronize()
        want = local.numpy()
        assert (want[0] != np.array([25, 25, 51], np.uint8)).any()
        comm = gpu.comm_init(1, 0, capi.comm_unique_id())
        slot = H * W * 3
        for scene_camera, rotate in ((False, False), (True, False), (True, True)):
            gpu.memset(frames.ptr, 0, frames.nbytes)
            gpu.gather_frames(comm, local.ptr, slot, frames.ptr, slot, S, H, W, scene_camera=scene_camera,
                              rotate_root=rotate)
            gpu.synchronize()
            assert np.array_equal(frames.numpy(), want), (scene_camera, rotate)
        with pytest.raises(capi.ErayError):  # rotating roots are a scene-camera transport
            gpu.gather_frames(comm, local.ptr, slot, frames.ptr, slot, S, H, W, rotate_root=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            gpu.gather_frames(comm, local.ptr, slot, frames.ptr, slot, S, H, W, scene_camera=True)
        gpu.memset(frames.ptr, 0, frames.nbytes)
        gpu.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(frames.numpy(), want), "graph replay"
    finally:
        if comm:
            capi.comm_destroy(comm)
        for a in (rgb, local, frames):
            a.free()
        sc.close()
        gpu.close()


@pytest.mark.parametrize("mesh", ["cube", "standin70k"])
def test_one_rank_gather_camera_path_frames(cube, standin70k_gather, mesh):
    """Camera-path frames through the scene-camera transport: the plan is the union of the path's
    cameras' pixel rectangles (accumulated on the device beside the path's setups), exchanged once
    per path call; the gathered frames equal the rendered ones.  Cube: batched setups (graph
    replay); 70k faces: the multi-camera builds."""
    import math
    W, H, S = 320, 180, 4
    gpu = capi.Context(0)
    sc = MainScene(gpu, *(cube if mesh == "cube" else standin70k_gather), W, H, texture=64, fov=(16.0, 9.0))
    ring = capi.frame_ring(S, H, W)
    rgb = gpu.empty((S, H, W, 3), np.float32)
    local = gpu.empty((S, H, W, 3), np.uint8)
    frames = gpu.empty((S, H, W, 3), np.uint8)
    comm = None
    try:
        path = [capi.make_camera((0.0, 0.0, 5.0 + 0.6 * math.sin(k)), (16.0, 9.0), W, 1.0 + 0.1 * k) for k in range(S)]
        gpu.render_camera_path(path, W, H, out_rgb=rgb.ptr, out_ppm=local.ptr, ring=ring)
        gpu.synchronize()
        want = local.numpy()
        assert all((want[k] != np.array([25, 25, 51], np.uint8)).any() for k in range(S))
        assert not np.array_equal(want[0], want[S - 1])  # the camera moved
        comm = gpu.comm_init(1, 0, capi.comm_unique_id())
        slot = H * W * 3
        for _ in range(2):  # (the second call reuses the path's plan)
            gpu.memset(frames.ptr, 0, frames.nbytes)
            gpu.gather_frames(comm, local.ptr, slot, frames.ptr, slot, S, H, W, scene_camera=True)
            gpu.synchronize()
            assert np.array_equal(frames.numpy(), want)
        # a second path into the same slots: a new plan, its own union
        path2 = [capi.make_camera((0.0, 0.0, 4.2 + 0.3 * k), (16.0, 9.0), W, 1.0) for k in range(S)]
        gpu.render_camera_path(path2, W, H, out_rgb=rgb.ptr, out_ppm=local.ptr, ring=ring)
        gpu.synchronize()
        want2 = local.numpy()
        gpu.memset(frames.ptr, 0, frames.nbytes)
        gpu.gather_frames(comm, local.ptr, slot, frames.ptr, slot, S, H, W, scene_camera=True)
        gpu.synchronize()
        assert np.array_equal(frames.numpy(), want2)
    finally:
        if comm:
            capi.comm_destroy(comm)
        for a in (rgb, local, frames):
            a.free()
        sc.close()
        gpu.close()


def test_scene_camera_gather_refuses_other_frames(cube):
    """The scene-camera transport only takes frames whose pixel rectangles it knows: frames this
    context did not render, anti-aliased frames (no rectangles), a batch mixing renders, and
    frames older than the context's latest scene-camera render, and a null `local` all fail with
    ERAY_E_INVALID_ARGUMENT (never a silently wrong frame); frames of the latest render still
    gather after each refusal."""
    W, H, S = 320, 180, 2
    gpu = capi.Context(0)
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    local = gpu.empty((S, H, W, 3), np.uint8)
    frames = gpu.empty((S, H, W, 3), np.uint8)
    other = gpu.empty((S, H, W, 3), np.uint8)
    slot = H * W * 3
    comm = None

    def gather(ptr, n=S):
        gpu.gather_frames(comm, ptr, slot, frames.ptr, slot, n, H, W, scene_camera=True)
        gpu.synchronize()

    def refused(ptr, n=S):
        with pytest.raises(capi.ErayError) as e:
            gather(ptr, n)
        assert e.value.status == capi.E_INVALID_ARGUMENT, e.value.message

    try:
        comm = gpu.comm_init(1, 0, capi.comm_unique_id())
        ring = capi.frame_ring(S, H, W)
        gpu.render_frames(S, W, H, out_ppm=local.ptr, ring=ring)
        gpu.synchronize()
        want = local.numpy()
        gather(local.ptr)
        assert np.array_equal(frames.numpy(), want)
        refused(other.ptr)  # never rendered by this context
        gpu.render(W, H, out_ppm=local.ptr, anti_aliasing=2, aa_seed=7)  # slot 0: anti-aliased
        refused(local.ptr)  # mixed: slot 0 anti-aliased, slot 1 the scene camera
        refused(local.ptr, 1)  # anti-aliased alone
        gpu.render_frames(S, W, H, out_ppm=local.ptr, ring=ring)
        gather(local.ptr)
        assert np.array_equal(frames.numpy(), want)
        # the scene camera moves and is rendered elsewhere: the plan follows the context's latest
        # render (state every rank shares), so the old frames are refused ...
        old_cam = capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0)  # (MainScene's camera)
        gpu.set_camera(capi.make_camera((0.0, 0.0, 4.0), (16.0, 9.0), W, 1.0))
        gpu.render(W, H, out_ppm=other.ptr)
        refused(local.ptr)
        gather(other.ptr, 1)  # the new camera's frame: a new plan
        assert np.array_equal(frames.numpy()[0], other.numpy()[0])
        refused(local.ptr)
        # ... until the old camera is rendered again (the same source key: its frames gather)
        gpu.set_camera(old_cam)
        gpu.render(W, H, out_ppm=other.ptr)
        gather(local.ptr)
        assert np.array_equal(frames.numpy(), want)
        # a null `local` is this rank's own error, after which the plan still serves
        refused(0)
        gather(local.ptr)
        assert np.array_equal(frames.numpy(), want)
    finally:
        if comm:
            capi.comm_destroy(comm)
        for a in (local, frames, other):
            a.free()
        sc.close()
        gpu.close()
