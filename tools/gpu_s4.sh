bash tools/gpu_round.sh s4 && bash tools/shard_sizes.sh shards2
