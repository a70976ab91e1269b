#!/usr/bin/env python3
"""Evaluate VELOCITY-ASR on an MI355X: transcribe a directory, or score WER/CER on a test set.

Same command line and printed report as the reference's scripts/evaluate.py:

    python scripts/evaluate.py --checkpoint model.pt --audio-dir ./test_audio [--output out.tsv]
    python scripts/evaluate.py --checkpoint model.pt --test-set manifest.tsv

--test-set takes a TSV manifest (`audio_path<TAB>reference text`); the reference's
dataset loader is a stub that loads nothing. --beam-width > 1 selects prefix beam search.
"""

import argparse
import logging
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from velocity_asr import VELOCITYASR, CTCDecoder, create_default_vocabulary  # noqa: E402
from velocity_asr.training import compute_cer, compute_wer  # noqa: E402
from velocity_asr.transcription import find_audio_files, load_manifest, transcribe_files  # noqa: E402

logging.basicConfig(level=logging.INFO, format="%(asctime)s | %(levelname)s | %(message)s",
                    datefmt="%Y-%m-%d %H:%M:%S")
logger = logging.getLogger("evaluate")

RULE = "=" * 60


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Evaluate VELOCITY-ASR v2 (MI355X)")
    p.add_argument("--checkpoint", required=True, help="Path to model checkpoint")
    p.add_argument("--test-set", default=None, help="Test-set manifest (TSV: audio path, reference)")
    p.add_argument("--audio-dir", default=None, help="Directory containing audio files to transcribe")
    p.add_argument("--output", default=None, help="Output file for results")
    p.add_argument("--device", default="cuda", help="HIP device to run evaluation on")
    p.add_argument("--beam-width", type=int, default=1, help="Beam width for decoding (1 = greedy)")
    p.add_argument("--batch-size", type=int, default=16, help="Max equal-length files per device batch")
    args = p.parse_args(argv)
    if args.test_set is None and args.audio_dir is None:
        p.error("Either --test-set or --audio-dir must be specified")
    return args


def main(argv=None) -> int:
    args = parse_args(argv)
    logger.info(f"Loading model from {args.checkpoint}")
    model = VELOCITYASR.from_pretrained(args.checkpoint)
    model.to(args.device)
    model.eval()
    logger.info(f"Model loaded with {model.count_parameters():,} parameters")
    decoder = CTCDecoder(create_default_vocabulary(model.config.vocab_size))

    if args.audio_dir:
        files = find_audio_files(args.audio_dir)
        rows = []
        for path, r in zip(files, transcribe_files(model, files, decoder, args.device, False,
                                                    args.batch_size, args.beam_width)):
            if "error" in r:
                logger.error(f"Error processing {path}: {r['error']}")
                rows.append((path.name, f"[ERROR: {r['error']}]"))
            else:
                rows.append((path.name, r["transcription"]))
        print("\n" + RULE)
        print("TRANSCRIPTION RESULTS")
        print(RULE)
        for name, text in rows:
            print(f"\n{name}:")
            print(f"  {text}")
        if args.output:
            with open(args.output, "w") as f:
                for name, text in rows:
                    f.write(f"{name}\t{text}\n")
            logger.info(f"Results saved to {args.output}")
        return 0

    data = load_manifest(args.test_set)
    if not data:
        logger.error("No test data loaded. Exiting.")
        return 0
    preds, refs = [], []
    results = transcribe_files(model, [a for a, _ in data], decoder, args.device, False,
                               args.batch_size, args.beam_width)
    for (audio, ref), r in zip(data, results):
        if "error" in r:
            logger.error(f"Error processing {audio}: {r['error']}")
            continue
        preds.append(r["transcription"])
        refs.append(ref)
    wer, cer = compute_wer(preds, refs), compute_cer(preds, refs)
    report = [f"Test Set: {args.test_set}", f"Samples: {len(preds)}",
              f"WER: {wer * 100:.2f}%", f"CER: {cer * 100:.2f}%"]
    print("\n" + RULE)
    print("EVALUATION RESULTS")
    print(RULE)
    print("\n".join(report))
    print(RULE)
    if args.output:
        with open(args.output, "w") as f:
            f.write("\n".join(report) + "\n")
        logger.info(f"Results saved to {args.output}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
