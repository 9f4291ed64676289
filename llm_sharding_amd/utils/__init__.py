"""Reference-compatible public API (module names and signatures of seanbonjean/llm-sharding's
``utils/`` package), implemented on the MI355X-native runtime:

  node_worker      Communicator, NodeWorker, NodeController
  config_sender    ConfigSender
  model_sharder    ModelSharder
  shard_loader     LlamaShardPart
  forwarding_utils build_position_ids
  node_profiler    NodeProfiler
  master_node      MasterNode (the scheduler the reference README describes but does not ship)
"""
