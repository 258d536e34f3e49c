"""experimental.shuffle (reference python/ray/tests/test_shuffle.py)."""
import numpy as np


def test_simple_shuffle_streaming_and_not(ray_shared):
    from ray_memory_management_amd.experimental import shuffle

    for no_streaming in (False, True):
        t, total = shuffle.run(num_partitions=4, partition_size=2e5, no_streaming=no_streaming, quiet=True)
        assert total == (int(2e5) // 16 // 4) * 4 * 16 * 4


def test_shuffle_merge_factor_and_items(ray_shared):
    from ray_memory_management_amd.experimental.shuffle import ObjectStoreWriterNonStreaming, simple_shuffle

    def reader(i):
        return iter(range(i * 10, i * 10 + 10))

    def writer(j, items):
        return sorted(items)

    out = simple_shuffle(input_reader=reader, input_num_partitions=6, output_num_partitions=3, output_writer=writer,
                         object_store_writer=ObjectStoreWriterNonStreaming, merge_factor=2)
    assert sorted(x for part in out for x in part) == list(range(60))
    assert [len(p) for p in out] == [24, 18, 18]  # round robin of 10 items per mapper over 3


def test_shuffle_with_tracker(ray_shared, capsys):
    from ray_memory_management_amd.experimental import shuffle

    tr = shuffle._StatusTracker.remote()
    shuffle.run(num_partitions=3, partition_size=1e5, tracker=tr, quiet=True, use_wait=True)
    assert "Reduce progress: 3/3" in capsys.readouterr().out
