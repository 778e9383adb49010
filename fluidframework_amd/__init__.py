"""MI355X-native batched merge-tree replay engine (drop-in for the observer path of
@fluidframework/merge-tree Client.applyMsg / Client.summarize)."""
