"""extract_map_objects.py (reference root): MapObjects.txt -> objects/<id>.npy + <id>.ply.

Same command line (-c config, -m map_dir, -n voxels_dim, default 128) on the device mesher
(reconstruct.map_objects.extract_map_objects over MeshExtractor).
"""
import argparse

from reconstruct.map_objects import extract_map_objects
from reconstruct.optimizer import MeshExtractor
from reconstruct.utils import get_configs, get_decoder


def config_parser():
    parser = argparse.ArgumentParser()
    parser.add_argument('-c', '--config', type=str, required=True, help='path to config file')
    parser.add_argument('-m', '--map_dir', type=str, required=True, help='path to map directory')
    parser.add_argument('-n', '--voxels_dim', type=int, default=128,
                        help='voxels resolution for running marching cube')
    return parser


if __name__ == "__main__":
    args = config_parser().parse_args()
    configs = get_configs(args.config)
    decoder = get_decoder(configs)
    extract_map_objects(args.map_dir, MeshExtractor(decoder, configs.optimizer.code_len, args.voxels_dim))
