"""CLI parsers — same flags as the reference's utils/parsers.py:5-31."""
import argparse


def training_argument_parser():
    parser = argparse.ArgumentParser(description="Experiment Args")
    parser.add_argument('-c', "--config-file", dest='config_file', required=True, help="path to config file")
    parser.add_argument('-p', "--project", dest='project', required=True, help="w&b project")
    parser.add_argument('-o', "--output-dir", dest='output_dir', required=True, help="path to output directory")
    parser.add_argument('-d', "--dataset-dir", dest='dataset_dir', default="", required=True,
                        help="path to dataset directory (synthetic pairs are generated when it holds no SpaceNet7 data)")
    parser.add_argument("opts", help="Modify config options using the command-line", default=None,
                        nargs=argparse.REMAINDER)
    return parser


def preprocess_argument_parser():
    parser = argparse.ArgumentParser(description="Experiment Args")
    parser.add_argument('-d', "--dataset", dest='dataset', required=True, help="path to dataset")
    parser.add_argument("opts", help="Modify config options using the command-line", default=None,
                        nargs=argparse.REMAINDER)
    return parser
