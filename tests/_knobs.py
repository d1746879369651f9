"""Kernel-selection helpers for the parity tests, over the C ABI's selection entry points
(ore_ctx_set_conv_tile, ore_ctx_set_pool_variant, ore_model_set_step_tile).  The library reads no
environment variables: a test picks kernels through the same calls a user would."""
import contextlib

# pooled-conv kernels (ore.Model.TILE_NAMES): EPOOL_TILE_BASE + variant, the window kernel, the f16
# one-launch first conv
EPOOL_TILE_BASE = 21
EPOOL_PATCH, EPOOL_WALK48, EPOOL_WALK96, EPOOL_WALK64, EPOOL_WALK64_B3 = 22, 23, 24, 25, 26
EPOOL_WINDOW = 44
C1_POOL_F16 = 43


@contextlib.contextmanager
def conv_tile(ctx, tile):
    """Every conv planned on ctx inside the block (per-op calls, models loaded) uses `tile` where its
    kernel family has it."""
    ctx.set_conv_tile(tile)
    try:
        yield
    finally:
        ctx.set_conv_tile(-1)


@contextlib.contextmanager
def pool_variant(ctx, variant):
    ctx.set_pool_variant(variant)
    try:
        yield
    finally:
        ctx.set_pool_variant(0)


def force_tiles(model, tile):
    """ore_model_set_step_tile(tile) on every exec step whose kernel family has it; returns how many.
    Call after set_fusion (re-planning renumbers the steps)."""
    import ore
    n = 0
    for i in range(len(model.tiles())):
        try:
            model.set_tile(i, tile)
            n += 1
        except ore.OreError:
            pass
    return n
