"""sdmi.streams: the engines' concurrent streams bound first, each on a hardware queue of its own (streams.py). After
reserve() the UNet engine takes exactly the reserved streams, in order (weight-gradient A, weight-gradient B,
context); a second engine gets fresh ones; and a trainer step on the reserved streams is bitwise the step of a trainer
on fresh streams (the queue placement changes timing only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_engine_takes_reserved_streams_in_order():
    from sdmi import streams
    from sdmi.trainer import DDPMTrainer
    from oracle import sd_oracle as O
    from tests.golden.configs import SMALL_COND
    dev = torch.device("cuda", 0)
    streams._RESERVED.clear()
    streams.reserve(dev, n=3)
    reserved = list(streams._RESERVED[0])
    assert len({s.cuda_stream for s in reserved}) == 3
    sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=7)
    a = DDPMTrainer(SMALL_COND, sd, dev, lr=1e-3)
    eng = a.engine
    assert [s.cuda_stream for s in (eng.sides[0], eng.sides[1], eng.ctx_stream)] == [s.cuda_stream for s in reserved]
    assert not streams._RESERVED[0]  # all taken
    b = DDPMTrainer(SMALL_COND, sd, dev, lr=1e-3)
    taken = {s.cuda_stream for s in reserved}
    assert not taken & {s.cuda_stream for s in (b.engine.sides[0], b.engine.sides[1], b.engine.ctx_stream)}
    g = torch.Generator().manual_seed(3)
    for s in range(2):
        x0 = torch.randn(2, 4, 32, 32, generator=g).cuda()
        noise = torch.randn(2, 4, 32, 32, generator=g).cuda()
        t = torch.randint(0, 1000, (2,), generator=g).cuda()
        text = torch.randn(2, 77, 64, generator=g).cuda()
        cmap = torch.randint(0, 19, (2, 64, 64), generator=g)
        mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float().cuda()
        a.step(x0, noise, t, text, mask)
        b.step(x0, noise, t, text, mask)
    a.sync_optimizer()
    b.sync_optimizer()
    torch.cuda.synchronize()
    assert torch.equal(a.store.params, b.store.params) and torch.equal(a.state, b.state)
