"""Host logic of the overlapped pipe runner (fused.overlap_bounds): the item
ranges that PipeRunner.run_overlapped / bench.py --pipe-parts launch."""
import pytest

from image_processor_pipeline_amd import fused


@pytest.mark.parametrize("n", [0, 1, 7, 8, 21, 4096, 4099])
@pytest.mark.parametrize("parts,ratio", [(1, 1.0), (2, 1.0), (3, 1.0), (5, 0.3), (16, 1.0), (40, 1.0), (4, 0.5)])
def test_bounds_cover_the_batch_in_whole_groups(n, parts, ratio):
    b = fused.overlap_bounds(n, parts, ratio, group=8)
    assert len(b) == parts + 1 and b[0] == 0 and b[-1] == n
    assert all(x <= y for x, y in zip(b, b[1:]))
    assert all(x % 8 == 0 or x == n for x in b)  # whole copy groups (the last one may be short)


def test_equal_and_geometric_shares():
    assert fused.overlap_bounds(4096, 3, 1.0, group=8) == [0, 1368, 2728, 4096]
    b = fused.overlap_bounds(4096, 2, 0.15, group=8)
    assert b[1] == 3560  # 1 / 1.15 of 512 groups


@pytest.mark.parametrize("args", [(-1, 2, 1.0), (8, 0, 1.0), (8, 2, 0.0)])
def test_bad_arguments(args):
    with pytest.raises(ValueError):
        fused.overlap_bounds(*args)
