"""C-ABI surface of libgr.so: loads, exports every symbol include/gr.h declares,
config struct layout matches the ctypes mirror.  No device compute here."""
import ctypes as C
import os
import re

import pytest

from generalizableracing_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gr_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_all_exports():
    assert declared_symbols() == sorted(_abi.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _abi.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_library_was_built_from_these_sources():
    """gr_source_sha256(): the in-tree libgr.so is the build of this tree's csrc sources (Makefile's SRCS + HDRS); a
    stale binary beside edited sources fails here instead of testing old kernels."""
    lib = _abi.load()
    assert lib.gr_source_sha256().decode() == _abi.tree_source_sha256()


def test_config_layout_and_defaults():
    lib = _abi.load()
    assert lib.gr_config_size() == C.sizeof(_abi.GrConfig)
    assert lib.gr_abi_version() == _abi.GR_ABI_VERSION
    c = _abi.default_config()
    assert c.num_envs == 2048 and c.num_types == 20 and c.num_levels == 10 and c.max_gates == 8
    assert c.max_episode_length == 200  # ceil(6.0 / 0.03)
    assert abs(c.step_dt - 0.03) < 1e-9 and c.decimation == 3
    assert list(c.rate_gain_p) == [35.0] * 3
    assert c.w_collision == -100.0 and c.w_success == 20.0 and c.w_bad_pose == -30.0


def test_create_destroy_and_bytes():
    lib = _abi.load()
    c = _abi.default_config()
    c.num_envs = 65536
    ctx = C.c_void_p()
    assert lib.gr_create(C.byref(c), C.byref(ctx)) == 0
    assert lib.gr_num_blocks(ctx) == 256
    r, w = C.c_int64(), C.c_int64()
    assert lib.gr_bytes_per_env_step(ctx, C.byref(r), C.byref(w)) == 0
    assert r.value == 256 and w.value == 290
    # calls before binding fail loudly with a message, never crash
    assert lib.gr_step(ctx, None, None) != 0
    assert b"bound" in lib.gr_last_error(ctx)
    assert lib.gr_destroy(ctx) == 0


def test_create_accepts_fewer_envs_than_terrain_columns():
    """IL assigns env i to column floor(i / (N / num_cols)): with N < num_cols some columns get no env."""
    lib = _abi.load()
    c = _abi.default_config()
    c.num_envs = 1
    ctx = C.c_void_p()
    assert lib.gr_create(C.byref(c), C.byref(ctx)) == 0
    assert lib.gr_num_blocks(ctx) == 1
    assert lib.gr_destroy(ctx) == 0


@pytest.mark.parametrize("field,value", [("num_envs", 0), ("num_types", 65), ("action_lag", 2), ("integrator", 7)])
def test_create_rejects_bad_config(field, value):
    lib = _abi.load()
    c = _abi.default_config()
    setattr(c, field, value)
    ctx = C.c_void_p()
    assert lib.gr_create(C.byref(c), C.byref(ctx)) == _abi.__dict__.get("GR_ERR_ARG", -1)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _abi.load(str(tmp_path / "libgr.so"))


def test_adam_prepare_numbers_blocks_and_rejects_bad_tables():
    """gr_adam_prepare (host only): block_start per segment in GR_ADAM_BLOCK = 1024 element blocks, the launch's
    block count; null pointers, empty segments and a shared step slot are argument errors; ctypes layout of the
    segment (48 B) and of the launch arguments (80 B) as in include/gr.h."""
    from generalizableracing_amd.rsl_rl.flat_adam import GrAdamArgs, GrAdamSegment

    assert C.sizeof(GrAdamSegment) == 48 and C.sizeof(GrAdamArgs) == 80
    lib = _abi.load()
    sizes = [4096, 256, 1, 1025, 3]
    t = (GrAdamSegment * len(sizes))()
    for i, n in enumerate(sizes):
        t[i].param = t[i].grad = t[i].exp_avg = t[i].exp_avg_sq = 0x1000
        t[i].numel, t[i].step_slot = n, len(sizes) - 1 - i
    nb = C.c_int32()
    assert lib.gr_adam_prepare(C.addressof(t), len(sizes), C.byref(nb)) == 0
    assert [t[i].block_start for i in range(len(sizes))] == [0, 4, 5, 6, 8]
    assert nb.value == 9
    t[3].step_slot = t[0].step_slot
    assert lib.gr_adam_prepare(C.addressof(t), len(sizes), C.byref(nb)) == -1  # GR_ERR_ARG
    t[3].step_slot = 1
    t[2].numel = 0
    assert lib.gr_adam_prepare(C.addressof(t), len(sizes), C.byref(nb)) == -1  # GR_ERR_ARG
    t[2].numel = 1
    t[1].grad = None
    assert lib.gr_adam_prepare(C.addressof(t), len(sizes), C.byref(nb)) == -1  # GR_ERR_ARG
    assert lib.gr_adam_prepare(C.addressof(t), 65, C.byref(nb)) == -1  # GR_ERR_ARG


def test_mlp_rejects_rows_past_32_bit_offsets():
    """gr_mlp_forward / _backward index rows * max(H, ldx) elements in 32 bits: a larger call is an argument error
    (checked before any launch; no device needed), whoever the caller is."""
    from generalizableracing_amd.rsl_rl.linear import GrMlpArgs, GrMlpNet

    lib = _abi.load()
    assert lib.gr_mlp_args_size() == C.sizeof(GrMlpArgs)
    a = GrMlpArgs()
    s = GrMlpNet()
    for name in ("x", "w1", "b1", "w2", "b2", "w3", "b3", "h1", "z2", "y", "gy", "gz2", "grads"):
        setattr(s, name, 0x10000)
    s.ldx, s.d, s.k = 16, 16, 4
    a.net[0] = s
    a.nets, a.hidden, a.slope, a.partial = 1, 256, 0.01, 0x10000
    for rows in (2 ** 31 // 256, 2 ** 40):  # rows * H = 2^31, and a row count past int32
        a.rows = rows
        assert lib.gr_mlp_forward(C.byref(a), None) == -1  # GR_ERR_ARG
        assert lib.gr_mlp_backward(C.byref(a), None) == -1
    a.rows, a.hidden = 2 ** 31 // 128 - 1, 128
    a.net[0].ldx = 160  # the strided input dominates: rows * ldx >= 2^31
    assert lib.gr_mlp_forward(C.byref(a), None) == -1


def test_stem12_rejects_shapes_it_does_not_cover():
    """gr_stem12_backward (the first block's backward with conv2's input gradient inside) covers 16 channels and table-a
    rows grouped as conv2's patches (na = 9 n2) with 16-byte aligned gz2 / w2t: anything else is an argument error,
    checked before any launch (no device needed)."""
    lib = _abi.load()
    p = 0x10000  # aligned dummy device pointers: the checks return before any launch

    def call(c=16, na=720, nb=48, n2=80, gz2=p, w2t=p, act=_abi.GR_POLICY_ACT_LRELU):
        return lib.gr_stem12_backward(p, 6928, 16, None, 8, p, na, nb, p, c, p, p, p, act, 0.01, gz2, n2, w2t, p, p, p, p,
                                      None)

    assert call(c=8) == -1
    assert call(na=721) == -1          # na != 9 n2
    assert call(n2=0, na=0) == -1
    assert call(gz2=p + 4) == -1       # gz2 not 16-byte aligned
    assert call(w2t=None) == -1
    assert call(act=7) == -1


def test_stem12_w2_backward_rejects_shapes_it_does_not_cover():
    """gr_stem12_backward_w2 (conv2's weight gradient inside the first block's backward) covers what gr_stem12_backward
    covers with at most 80 conv2 patches per image (its offsets live in registers) and a gw2 output; anything else is
    an argument error before any launch.  Its workspace: per workgroup (<= 256) the BN, conv1 and conv2 partials."""
    lib = _abi.load()
    p = 0x10000

    def call(c=16, na=720, nb=48, n2=80, gz2=p, w2t=p, gw2=p, act=_abi.GR_POLICY_ACT_LRELU, mom=None):
        return lib.gr_stem12_backward_w2(p, 6928, 16, None, 8, p, na, nb, p, c, p, p, p, mom, act, 0.01, gz2, n2, w2t,
                                         p, p, p, gw2, p, None)

    assert call(c=8) == -1
    assert call(n2=81, na=729) == -1   # past the 80 patches the kernel holds
    assert call(na=721) == -1
    assert call(gz2=p + 4) == -1
    assert call(gw2=None) == -1
    assert call(act=7) == -1
    assert call(mom=p + 4) == -1  # (the forward's moments: 8-byte aligned doubles, or null)
    assert lib.gr_stem12_backward_w2_scratch_doubles(0) == -1
    assert lib.gr_stem12_backward_w2_scratch_doubles(1) == 32 + 16 + 432 + 4608
    assert lib.gr_stem12_backward_w2_scratch_doubles(24576) == 256 * (32 + 432 + 4608) + 16


def test_stem12_forward_rejects_shapes_it_does_not_cover():
    """gr_stem12_forward (conv2 inside the first block's apply pass): 16 channels, na = 9 n2, 16-byte aligned outputs
    and weights; anything else is an argument error before any launch."""
    lib = _abi.load()
    p = 0x10000

    def call(c=16, na=720, n2=80, w2f=p, z2=p, act=_abi.GR_POLICY_ACT_LRELU, mom=None):
        return lib.gr_stem12_forward(p, 6928, 16, None, 8, p, na, 48, p, c, p, p, 1e-5, act, 0.01, w2f, n2, p, z2, p, mom,
                                     p, None)

    assert call(c=32) == -1
    assert call(na=718) == -1
    assert call(w2f=p + 8) == -1
    assert call(z2=None) == -1
    assert call(act=5) == -1
    assert call(mom=p + 4) == -1


def test_patch_wgrad_rejects_shapes_it_does_not_cover():
    """gr_patch_wgrad (the stem's conv2 / conv3 / Linear weight gradients): n 32 with k 128 or 144, n a multiple of
    64 up to 256 with k a multiple of 128 up to 4096; ld >= k; 16-byte aligned gy, 4-byte aligned x; m >= 1."""
    lib = _abi.load()
    p = 0x10000
    assert lib.gr_patch_wgrad_floats(4096, 32, 144) > 0
    assert lib.gr_patch_wgrad_floats(491520, 64, 128) > 0
    assert lib.gr_patch_wgrad_floats(24576, 192, 1280) > 0
    assert lib.gr_patch_wgrad_floats(24576, 96, 128) == -1
    assert lib.gr_patch_wgrad_floats(1, 32, 100) == -1
    assert lib.gr_patch_wgrad_floats(100, 64, 144) == -1
    assert lib.gr_patch_wgrad_floats(0, 32, 144) == -1

    def call(x=p, ld=144, gy=p, m=100, n=32, k=144):
        return lib.gr_patch_wgrad(x, ld, gy, m, n, k, p, p, None)

    assert call(k=64) == -1
    assert call(n=48) == -1
    assert call(m=0) == -1
    assert call(ld=100) == -1
    assert call(x=p + 2) == -1
    assert call(gy=p + 4) == -1
    assert call(gy=None) == -1


def test_bn_running_update_rejects_bad_arguments():
    """gr_bn_running_update: non-null running buffers and stats, 1 <= c <= 4096, uses >= 1, a batch count needs its
    counter."""
    lib = _abi.load()
    p = 0x10000

    def call(rm=p, nbt=p, c=16, uses=1, count=1):
        return lib.gr_bn_running_update(rm, p, nbt, p, c, 0.9, 0.1, uses, count, None)

    assert call(rm=None) == -1
    assert call(c=0) == -1
    assert call(uses=0) == -1
    assert call(nbt=None) == -1
    assert call(count=-1) == -1


def test_tsgemm_rejects_shapes_it_does_not_cover():
    """gr_tsgemm: (k 128, n 64, b as [n][k]) or (k 64, n 128, b as [k][n]); lda >= k, ldc >= n; 4-byte aligned A."""
    lib = _abi.load()
    p = 0x10000

    def call(a=p, lda=128, b_nk=1, ldc=64, m=100, k=128, n=64):
        return lib.gr_tsgemm(a, lda, p, b_nk, p, ldc, m, k, n, None)

    assert call(m=0) == 0
    assert call(b_nk=0) == -1
    assert call(k=64, n=128, lda=64, ldc=128) == -1
    assert call(n=32) == -1
    assert call(k=192, n=100, b_nk=0, lda=192, ldc=100) == -1
    assert call(lda=100) == -1
    assert call(ldc=32) == -1
    assert call(a=p + 2) == -1
    assert call(a=None) == -1


def test_l2c2_mix_rows_rejects_bad_arguments():
    """gr_l2c2_mix_rows: both row-index arrays, cols a multiple of 4, ld >= cols and a multiple of 4, 16-byte aligned
    sources and output."""
    lib = _abi.load()
    p = 0x10000

    def call(ra=p, ld=6928, cols=6928, out=p):
        return lib.gr_l2c2_mix_rows(p, p, ld, ra, p, p, 8, cols, out, None)

    assert call(ra=None) == -1
    assert call(cols=6926) == -1
    assert call(ld=6000) == -1
    assert call(ld=6930) == -1
    assert call(out=p + 4) == -1
