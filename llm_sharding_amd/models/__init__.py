"""Model definitions: config-driven Llama decoder, golden reference, RoPE, shard IO, tokenizer."""
