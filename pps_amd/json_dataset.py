"""Re-ID dataset ingestion: the COCO-style json that tools/bpm_to_coco.py
writes, read without pycocotools.

Reference behaviour reproduced (detectron/datasets/json_dataset.py):
  * image ids sorted ascending (:106-108); roidb entry `image` = image_directory
    + image_prefix + file_name (:142-147);
  * exactly one annotation per image, carrying `mark` (0 = query, 1 = gallery,
    2 = multi-query) (:188-189; written by tools/bpm_to_coco.py:147);
  * dataset name -> (image dir, annotation file) catalog
    (detectron/datasets/dataset_catalog.py:205-240), rooted at
    $PPS_DATA_DIR (the reference's _DATA_DIR).
Person id / camera are parsed from the file name by the evaluator
(reid_dataset_evaluator.py:212-231: id = name[:8], cam = name[9:13]).
"""
import json
import os

DATA_DIR = os.environ.get('PPS_DATA_DIR', os.path.join(os.getcwd(), 'data'))

# name -> (image directory, annotation file), relative to DATA_DIR
CATALOG = {
    'market1501_trainval': ('market1501/images', 'market1501/trainval.json'),
    'market1501_test': ('market1501/images', 'market1501/test.json'),
    'duke_trainval': ('duke/images', 'duke/trainval.json'),
    'duke_test': ('duke/images', 'duke/test.json'),
    'cuhk03_trainval': ('cuhk03/labeled/images', 'cuhk03/labeled/trainval.json'),
    'cuhk03_test': ('cuhk03/labeled/images', 'cuhk03/labeled/test.json'),
    # BASELINE.json configs[3] asks for the detected split; the reference
    # catalog only lists labeled (dataset_catalog.py:235-240).
    'cuhk03_detected_test': ('cuhk03/detected/images', 'cuhk03/detected/test.json'),
}


def dataset_paths(name):
    if os.path.isfile(name):  # a json path given directly
        return os.path.dirname(os.path.abspath(name)), name
    if name not in CATALOG:
        raise KeyError('Unknown dataset name: %s' % name)
    im_dir, ann = CATALOG[name]
    return os.path.join(DATA_DIR, im_dir), os.path.join(DATA_DIR, ann)


class JsonDataset(object):
    def __init__(self, name, image_directory=None, annotation_file=None, image_prefix=''):
        self.name = name
        if annotation_file is None:
            image_directory, annotation_file = dataset_paths(name)
        self.image_directory = image_directory
        self.annotation_file = annotation_file
        self.image_prefix = image_prefix
        with open(annotation_file) as f:
            self.coco = json.load(f)
        self._ann_by_image = {}
        for a in self.coco.get('annotations', []):
            self._ann_by_image.setdefault(a['image_id'], []).append(a)

    def get_roidb(self, gt=False, check_exists=False):
        images = sorted(self.coco['images'], key=lambda im: im['id'])
        roidb = []
        for im in images:
            path = os.path.join(self.image_directory, self.image_prefix + im['file_name'])
            if check_exists:
                assert os.path.exists(path), "Image '{}' not found".format(path)
            e = dict(id=im['id'], image=path, width=im.get('width'),
                     height=im.get('height'), mark=None)
            if gt:
                anns = self._ann_by_image.get(im['id'], [])
                assert len(anns) == 1, 'expected one annotation per image (json_dataset.py:187)'
                e['mark'] = anns[0].get('mark')
            roidb.append(e)
        return roidb


def write_coco_json(path, file_names, marks, sizes=None):
    """Minimal writer of the bpm_to_coco.py json layout (images + one
    annotation per image with `mark`), for synthetic / user datasets."""
    images, anns = [], []
    for i, (fn, mk) in enumerate(zip(file_names, marks)):
        w, h = sizes[i] if sizes is not None else (64, 128)
        images.append(dict(id=i + 1, file_name=fn, width=w, height=h))
        anns.append(dict(id=i + 1, image_id=i + 1, category_id=int(fn[:8]), mark=int(mk),
                         iscrowd=0, area=float(w * h), bbox=[0, 0, w, h]))
    with open(path, 'w') as f:
        json.dump(dict(images=images, annotations=anns, categories=[]), f)
