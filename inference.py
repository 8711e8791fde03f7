"""Entry point with the reference's command line (inference.py of StableAvatar, flags :238-409):
    python inference.py --config_path=deepspeed_config/wan2.1/wan_civitai.yaml --pretrained_model_name_or_path=...
Runs stableavatar_amd.inference.main on the MI355X HIP modules; under torchrun with
--ulysses_degree x --ring_degree > 1 it runs sequence parallel over RCCL."""
import sys

from stableavatar_amd.inference import main

if __name__ == "__main__":
    main()
    sys.exit(0)
