#!/usr/bin/env python3
"""Transcribe audio files with VELOCITY-ASR on an MI355X.

Same command line and outputs as the reference's scripts/transcribe.py:

    python scripts/transcribe.py audio.wav --checkpoint model.pt [--timestamps] [--format json]
    python scripts/transcribe.py --input-dir ./audio --output-dir ./out --checkpoint model.pt

Files of equal length are transcribed together as one device batch (--batch-size).
"""

import argparse
import json
import logging
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from velocity_asr import VELOCITYASR, CTCDecoder, create_default_vocabulary  # noqa: E402
from velocity_asr.transcription import find_audio_files, transcribe_files  # noqa: E402

logging.basicConfig(level=logging.INFO, format="%(asctime)s | %(levelname)s | %(message)s",
                    datefmt="%Y-%m-%d %H:%M:%S")
logger = logging.getLogger("transcribe")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Transcribe audio with VELOCITY-ASR v2 (MI355X)")
    p.add_argument("audio", nargs="?", default=None, help="Path to audio file")
    p.add_argument("--checkpoint", required=True, help="Path to model checkpoint")
    p.add_argument("--input-dir", default=None, help="Directory of audio files for batch transcription")
    p.add_argument("--output-dir", default=None, help="Output directory for per-file transcripts")
    p.add_argument("--output", "-o", default=None, help="Output file path")
    p.add_argument("--format", choices=["text", "json"], default="text", help="Output format")
    p.add_argument("--timestamps", action="store_true", help="Include word-level timestamps")
    p.add_argument("--device", default="cuda", help="HIP device to run inference on")
    p.add_argument("--quiet", "-q", action="store_true", help="Suppress logging output")
    p.add_argument("--batch-size", type=int, default=16, help="Max equal-length files per device batch")
    args = p.parse_args(argv)
    if args.audio is None and args.input_dir is None:
        p.error("Either audio file or --input-dir must be specified")
    return args


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.quiet:
        logging.getLogger().setLevel(logging.WARNING)

    logger.info(f"Loading model from {args.checkpoint}")
    model = VELOCITYASR.from_pretrained(args.checkpoint)
    model.to(args.device)
    model.eval()
    decoder = CTCDecoder(create_default_vocabulary(model.config.vocab_size))

    if args.input_dir:
        files = find_audio_files(args.input_dir)
        if not files:
            logger.error(f"No audio files found in {args.input_dir}")
            return 0
        logger.info(f"Found {len(files)} audio files")
        if args.output_dir:
            os.makedirs(args.output_dir, exist_ok=True)
        results = []
        for path, r in zip(files, transcribe_files(model, files, decoder, args.device, args.timestamps,
                                                    args.batch_size)):
            if "error" in r:
                logger.error(f"Error processing {path}: {r['error']}")
                continue
            results.append(r)
            if args.output_dir:
                out = Path(args.output_dir) / (path.stem + (".json" if args.format == "json" else ".txt"))
                with open(out, "w") as f:
                    if args.format == "json":
                        json.dump(r, f, indent=2)
                    else:
                        f.write(r["transcription"])
            if not args.quiet:
                print(f"\n{path.name}:")
                print(f"  {r['transcription']}")
        if args.output:
            with open(args.output, "w") as f:
                if args.format == "json":
                    json.dump(results, f, indent=2)
                else:
                    for r in results:
                        f.write(f"{r['file']}\t{r['transcription']}\n")
        logger.info(f"Processed {len(results)} files")
        return 0

    r = transcribe_files(model, [args.audio], decoder, args.device, args.timestamps, 1)[0]
    if "error" in r:
        logger.error(f"Error processing {args.audio}: {r['error']}")
        return 1
    text = json.dumps(r, indent=2) if args.format == "json" else r["transcription"]
    if args.output:
        with open(args.output, "w") as f:
            f.write(text)
        logger.info(f"Transcript saved to {args.output}")
    else:
        print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
