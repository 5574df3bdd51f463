import sys; sys.path[:0]=['streaming-zero-knowledge-proofs_amd']
import sezkp_amd as S
b=S.synthetic_blocks(4096,512,8,42)
try: S.StarkV1.prove(b, b.manifest_root()); print("ok")
except Exception as e: print("ERR", e)
