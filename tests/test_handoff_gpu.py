"""The persistent kernels' in-launch publication primitive (csrc/persist.h, used by
csrc/resident.hip, hybrid.hip and vanilla.hip), stress-tested word by word on the GPU
(csrc/handoff.hip): producers on every XCD rewrite a payload IN PLACE every round (as the
vanilla epoch's fc1 tiles are rewritten between its update and forward passes), consumers
re-read the same addresses every round (L1 / L2 warm with the previous round's value), random
per-round delays and a bandwidth stream on a random half of the workgroups make the load
uneven (MI355X_MICROARCH.md: "test every hand-off under UNEVEN load, consumer L1-warm,
checking every word").

* mode 0, the shipped form (sc1 stores, drained, one agent-scope counter add per workgroup;
  sc1 poll, workgroup barrier, sc1 loads): no stale word;
* mode 3, the LLVM AMDGPU memory model's fence form (plain stores, agent release before the
  add, agent acquire after the poll, plain loads) and mode 4 (shipped + acquire): no stale word;
* mode 1, plain stores and loads with no fences (the negative control): stale words ARE seen,
  so the test can detect the failure it guards against."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(mode, P=1024, nsrc=4, stride=37, R=1000, busy_us=4.0):
    from splitlearning_amd import _native
    C = _native.load()
    nbad, rmin, err, ms, first = C.handoff_stress(256, P, R, nsrc, stride, mode, busy_us, 10.0)
    assert err == 0 and rmin == R, (mode, err, rmin)
    return nbad, first


@pytest.mark.parametrize("mode", [0, 3, 4])
@pytest.mark.parametrize("P,nsrc,stride", [(1024, 4, 37), (256, 8, 9)])
def test_publication_primitive_never_stale(cuda, mode, P, nsrc, stride):
    nbad, first = _run(mode, P, nsrc, stride)
    assert nbad == 0, f"mode {mode}: {nbad} stale words, first {first}"


def test_negative_control_sees_stale_words(cuda):
    nbad, _ = _run(1)
    assert nbad > 0
